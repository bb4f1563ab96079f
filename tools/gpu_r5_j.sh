# round 5 call J: walk_stage (probe_walk1: the ordered walk, the duplicate-key partitioned walk)
# with 16-byte key loads — its tests, then A/B against the 8-byte form on the ordered C2 path
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_probe_gpu.py tests/test_pipeline_device_gpu.py \
  tests/test_known_answers_gpu.py tests/test_facade_gpu.py -k "ordered or partitioned or walk or reference_sum or pipeline" > gpurun_out/r5j_tests.log 2>&1 && \
bash tools/gpu_ab.sh r5ws c2ord 3 product tools/abx/libccj_ws8.so > gpurun_out/r5ws_ab.log 2>&1
