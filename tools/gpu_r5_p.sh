# round 5 call P: owner_split_direct with wave images — multi-GPU tests, then owner split alone:
# product vs the previous build (interleaved 3x), the imageless form and grid sizes (tuning build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py > gpurun_out/r5p_tests.log 2>&1 && \
o=gpurun_out/r5p_owner.log && : > $o && \
for i in 1 2 3; do
  echo "== product $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --unmasked >> $o 2>&1 && \
  echo "== own1 $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --lib tools/abx/libccj_own1.so --unmasked >> $o 2>&1 || exit 1
done && \
for v in CCJ_OWNER_DIRECT=1 CCJ_OWNER_DIRECT_PER_CU=4 CCJ_OWNER_DIRECT_PER_CU=6 CCJ_OWNER_ABLATE=48 CCJ_OWNER_ABLATE=1048576; do
  echo "== $v" >> $o && env $v timeout -k 10 120 python3 -u tools/owner_split_bench.py --lib tuning --unmasked >> $o 2>&1 || exit 1
done
