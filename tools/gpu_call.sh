# round 5 call BA: gather_payload_cols<8> with per-lane position loads shared to the quads by
# ds_bpermute (U / 4 = 2 position loads per wave and step instead of 8) against the product; C5 tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5ba c5 3 product tools/abx/libccj_gpos.so > gpurun_out/r5ba_ab.log 2>&1 && \
CCJ_LIB_PATH=tools/abx/libccj_gpos.so timeout -k 10 300 \
  python -u -m pytest tests/test_c5_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ba_tests.log 2>&1
