# round 5 call K: the C3 filter walks with 16-byte key loads — chaining tests, then A/B on C3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_probe_gpu.py tests/test_c3_gpu.py \
  tests/test_known_answers_gpu.py tests/test_build_gpu.py tests/test_bench_gpu.py -k "chain or c3 or reference_sum or build" > gpurun_out/r5k_tests.log 2>&1 && \
bash tools/gpu_ab.sh r5f16 c3split 3 product tools/abx/libccj_f8.so > gpurun_out/r5f16_ab.log 2>&1 && \
bash tools/gpu_r5_l.sh
