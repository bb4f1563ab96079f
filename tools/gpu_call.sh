# round 5 call AY: transposed-store gather step size at full occupancy — 512 rows (U=8, 5 WG/CU),
# 384 (U=6, 6 WG/CU), 256 (U=4, 8 WG/CU), tuning build; C5 tests on U=6 and U=4
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5ay c5 3 tuning tuning:CCJ_GATHER_U=6 tuning:CCJ_GATHER_U=4 > gpurun_out/r5ay_ab.log 2>&1 && \
for u in 6 4; do CCJ_LIB_PATH=chunk-compaction-in-vectorized-execution-simd_amd/libccj_tuning.so CCJ_GATHER_U=$u timeout -k 10 300 \
  python -u -m pytest tests/test_c5_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5ay_tests_$u.log 2>&1 || exit 1; done
