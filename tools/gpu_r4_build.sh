# round 4: device chaining build, work accounting, reference vectors on the GPU, then the GPU suite,
# then the facade micro-bench known answer (long: 8 x 2^19 one-chunk facade probes)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 120 ./tools/copybench 4 > gpurun_out/r4_copybench.log 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_build_gpu.py tests/test_cost_gpu.py tests/test_known_answers_gpu.py -x -v --timeout 300 --timeout-method thread -k "not micro_bench" --durations=10 > gpurun_out/r4_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_known_answers_gpu.py::test_micro_bench_known_answer_through_facade --durations=15 > gpurun_out/r4_suite.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_known_answers_gpu.py -x -v --timeout 280 --timeout-method thread -k micro_bench --durations=5 > gpurun_out/r4_micro.log 2>&1
