# round 5 call AC: the ordered route's walk as probe_walk2<MM> (fixed first windows, round words)
# — ordered / known-answer / pipeline / facade tests, then C2 ordered against the probe_walk1 build
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_probe_gpu.py tests/test_known_answers_gpu.py \
  tests/test_pipeline_device_gpu.py tests/test_facade_gpu.py -k "ordered or reference_sum or pipeline or facade or known" > gpurun_out/r5ac_tests.log 2>&1 && \
bash tools/gpu_ab.sh r5ow c2ord 3 product tools/abx/libccj_w1.so > gpurun_out/r5ow_ab.log 2>&1
