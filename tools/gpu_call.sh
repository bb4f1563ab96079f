# round 5 call BG: gather_payload_cols with its LDS tile XOR-swizzled (conflict-free 8-byte writes)
# against the product; C5 tests on it
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5bg c5 3 product tools/abx/libccj_gswz.so > gpurun_out/r5bg_ab.log 2>&1 && \
CCJ_LIB_PATH=tools/abx/libccj_gswz.so timeout -k 10 300 \
  python -u -m pytest tests/test_c5_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5bg_tests.log 2>&1
