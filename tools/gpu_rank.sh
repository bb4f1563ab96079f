# rank walk: new parity tests, the partitioned-probe tests, then the C2 bench (rank vs slot walk A/B)
# and a kernel trace of the same command
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_rank_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/rank_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-other --no-cpu > gpurun_out/bench_rank.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/kt_rank -o kt -- python3 bench.py --no-other --no-cpu --no-verify --steps 5 > gpurun_out/kt_rank.log 2>&1
