# round 5 call W: owner_split_direct with 16-byte key loads — multi-GPU tests, then owner split
# alone against the previous build (interleaved 3x)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r5w_tests.log 2>&1 && \
o=gpurun_out/r5w_owner.log && : > $o && \
for i in 1 2 3; do
  echo "== product $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --unmasked >> $o 2>&1 && \
  echo "== k8 $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --lib tools/abx/libccj_k8.so --unmasked >> $o 2>&1 || exit 1
done
