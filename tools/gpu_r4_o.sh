# round 4 call O: compaction with the join-key column filled from the payload (key_cols): compaction
# tests, C3 bench line (gathered form timed beside)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_compact_gpu.py tests/test_c3_gpu.py tests/test_abi_cpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 && \
timeout -k 10 240 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4o_c3.log 2>&1 && \
timeout -k 10 240 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4o_c3ord.log 2>&1
