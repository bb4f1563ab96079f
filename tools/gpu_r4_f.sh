# round 4 call F: filter walk v3 (batched chain rounds, key prefetch, 2 x 768-thread workgroups per
# CU): chain tests, C3 partitioned + ordered bench lines (kernel trace of the partitioned one), C2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 120 ./tools/storebench > gpurun_out/r4f_storebench.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3" > gpurun_out/r4f_tests.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4f_c3.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4f_c3ord.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r4f_c3kt -o kt -- python3 bench.py --workload c3 --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/r4f_c3kt.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4f_c2.log 2>&1
