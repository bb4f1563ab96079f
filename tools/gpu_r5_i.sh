# round 5 call I: probe_walk2 staging keys with 16-byte loads — the partitioned / known-answer /
# C5 tests (tuning build too: its DPP self-check), then A/B against the 8-byte form on C2 and C5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_probe_gpu.py tests/test_c5_gpu.py \
  tests/test_known_answers_gpu.py tests/test_rank_gpu.py -k "partitioned or walk or c5 or reference_sum or rank" > gpurun_out/r5i_tests.log 2>&1 && \
bash tools/gpu_ab.sh r5k16 c2 3 product tools/abx/libccj_k8.so > gpurun_out/r5k16_ab.log 2>&1 && \
bash tools/gpu_ab.sh r5k16c5 c5 2 product tools/abx/libccj_k8.so > gpurun_out/r5k16c5_ab.log 2>&1
