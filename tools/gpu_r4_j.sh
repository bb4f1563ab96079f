# round 4 call J: filter walk v4 + first-match exit: chain tests, C3 bench; C3 at chain window bits
# 17 (512 partitions, tuning build) to separate the split's partition count from its key skew
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3" > gpurun_out/r4j_tests.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4j_c3.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4j_c3ord.log 2>&1 && \
CCJ_WINDOW_BITS=18 timeout -k 10 180 python -u bench.py --lib tuning --workload c3 --no-cpu --no-verify --steps 10 --warmup 3 > gpurun_out/r4j_c3_wb17.log 2>&1 && \
timeout -k 10 180 python -u bench.py --lib tuning --workload c3 --no-cpu --no-verify --steps 10 --warmup 3 > gpurun_out/r4j_c3_tuning.log 2>&1
