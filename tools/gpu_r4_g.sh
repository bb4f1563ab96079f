# round 4 call G: the whole GPU test suite, then call C's multi-GPU rehearsal (C2 on the 2^27-key
# per-GPU table; one-rank sharded steps with local probes over groups of 16 and 32 batches)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4g_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --n-build 134217728 --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4g_c2_2e27.log 2>&1 && \
timeout -k 10 400 python -u bench.py --sharded --group 16 --no-cpu --steps 5 --warmup 2 > gpurun_out/r4g_sharded_g16.log 2>&1 && \
timeout -k 10 400 python -u bench.py --sharded --group 32 --no-cpu --steps 5 --warmup 2 > gpurun_out/r4g_sharded_g32.log 2>&1
