# round 5 call N: owner split with bit-sliced ballot ranking and the high-word hash — multi-GPU tests,
# then owner split alone, product vs the previous build (interleaved 3x)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r5n_tests.log 2>&1 && \
o=gpurun_out/r5n_owner.log && : > $o && \
for i in 1 2 3; do
  echo "== product $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --unmasked >> $o 2>&1 && \
  echo "== own0 $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --lib tools/abx/libccj_own0.so --unmasked >> $o 2>&1 || exit 1
done
