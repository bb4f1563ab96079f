# round 4 call H: filter walk v4 (scalar unit arithmetic, packed chain-row queue): chain tests, C3
# partitioned + ordered bench lines, kernel trace of the partitioned one
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3" > gpurun_out/r4h_tests.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4h_c3.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4h_c3ord.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r4h_c3kt -o kt -- python3 bench.py --workload c3 --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/r4h_c3kt.log 2>&1
