# round 5 call Q: the one-rank N > 1 rehearsal with owner_split_direct (groups of 32), the gfx950
# counter list (for a counter-backed pass naming the unit each C2 kernel waits on)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u bench.py --gpus 1 --sharded --group 32 --no-cpu > gpurun_out/r5q_sharded_g32.log 2> gpurun_out/r5q_sharded_g32.err && \
timeout -k 10 120 rocprofv3 -L > gpurun_out/r5q_counters.txt 2>&1
