# round 5 call AE: the split's overflow area in 4 sub-areas per XCD group, each with its own cursor
# line — partitioned / C3 / ordered / multi-GPU / known-answer tests, then C3 and C2 against the
# one-cursor-per-group build (interleaved)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_probe_gpu.py tests/test_c3_gpu.py \
  tests/test_dist_gpu.py tests/test_known_answers_gpu.py tests/test_c5_gpu.py > gpurun_out/r5ae_tests.log 2>&1 && \
bash tools/gpu_ab.sh r5ovc c3 3 product tools/abx/libccj_s1.so > gpurun_out/r5ovc_ab.log 2>&1 && \
bash tools/gpu_ab.sh r5ovc2 c2 2 product tools/abx/libccj_s1.so > gpurun_out/r5ovc2_ab.log 2>&1
