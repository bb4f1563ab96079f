# round 5 call AZ: transposed-store gather with two row buffers (step i + 2's rows in flight while
# step i stores; 114 VGPRs, 4 WG/CU) against one (5 WG/CU), tuning build; C5 tests on it
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5az c5 3 tuning tuning:CCJ_GATHER_T=2 > gpurun_out/r5az_ab.log 2>&1 && \
CCJ_LIB_PATH=chunk-compaction-in-vectorized-execution-simd_amd/libccj_tuning.so CCJ_GATHER_T=2 timeout -k 10 300 \
  python -u -m pytest tests/test_c5_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5az_tests.log 2>&1
