# round 4 call A: copy ceiling, the new build / cost / reference-vector tests, the chaining filter
# walks' tests, the C3 and C2 bench lines
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 120 ./tools/copybench 4 > gpurun_out/r4_copybench.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_build_gpu.py tests/test_cost_gpu.py tests/test_known_answers_gpu.py tests/test_probe_gpu.py -x -v --timeout 300 --timeout-method thread -k "not micro_bench and (chain or build or cost or reference_sum)" --durations=10 > gpurun_out/r4_new.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4_c3ord.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu --no-other --steps 10 --warmup 3 > gpurun_out/r4_c2.log 2>&1
