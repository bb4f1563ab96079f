# round 5 call X: the hand-written device scan in place of hipCUB's (compactor, pipeline, exact
# multisplit, chaining build) — its tests and every test of the paths that take offsets from it,
# then C3 (its timed compaction) against the previous build, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scan_gpu.py tests/test_compact_gpu.py \
  tests/test_c3_gpu.py tests/test_pipeline_gpu.py tests/test_pipeline_device_gpu.py tests/test_build_gpu.py tests/test_dist_gpu.py \
  tests/test_known_answers_gpu.py tests/test_probe_gpu.py > gpurun_out/r5x_tests.log 2>&1 && \
bash tools/gpu_ab.sh r5scan c3 2 product tools/abx/libccj_k8.so > gpurun_out/r5scan_ab.log 2>&1
