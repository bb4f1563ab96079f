# round 4 call M: per-XCD overflow sub-areas (the split's skewed runs reserve from their group's own
# cursor): partitioned / ordered / chain / dist-rank tests, split under three streams, C3 + C2 lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py tests/test_rank_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4m_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/exp_split_c3.py > gpurun_out/r4m_split.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4m_c3.log 2>&1 && \
timeout -k 10 180 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4m_c3ord.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu --no-other --steps 10 --warmup 3 > gpurun_out/r4m_c2.log 2>&1
