# round 4 call C: the single-GPU C2 path on the C4 per-GPU table (2^27 build keys), then the one-rank
# multi-GPU rehearsal with local probes over groups of 16 batches (two sweeps per step) and of all 32
# (one sweep)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u bench.py --n-build 134217728 --no-cpu --no-other --no-verify --steps 8 --warmup 2 > gpurun_out/r4c_c2_2e27.log 2>&1 && \
timeout -k 10 400 python -u bench.py --sharded --group 16 --no-cpu --steps 5 --warmup 2 > gpurun_out/r4c_sharded_g16.log 2>&1 && \
timeout -k 10 400 python -u bench.py --sharded --group 32 --no-cpu --steps 5 --warmup 2 > gpurun_out/r4c_sharded_g32.log 2>&1
