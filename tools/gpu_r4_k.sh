# round 4 call K: split with per-workgroup full-segment flags (skewed runs reserved in the overflow
# area once per wave, beside the segment reservations): partitioned / ordered / chain tests, C3 and
# C2 bench lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 500 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3 or partitioned or ordered" > gpurun_out/r4k_tests.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4k_c3.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4k_c3ord.log 2>&1 && \
CCJ_WINDOW_BITS=18 timeout -k 10 180 python -u bench.py --lib tuning --workload c3 --no-cpu --no-verify --steps 10 --warmup 3 > gpurun_out/r4k_c3_wb17.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu --no-other --steps 10 --warmup 3 > gpurun_out/r4k_c2.log 2>&1
