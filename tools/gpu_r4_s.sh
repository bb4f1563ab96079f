# round 4 call S: smoke, dist GPU tests, the one-rank rehearsal with the local probe timed alone,
# C5 and C2-ordered bench lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4s_smoke.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4s_dist.log 2>&1 && \
timeout -k 10 400 python -u bench.py --sharded --group 32 --no-cpu --steps 5 --warmup 2 > gpurun_out/r4s_sharded_g32.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu --steps 5 --warmup 2 > gpurun_out/r4s_c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --path ordered --no-cpu --no-other --steps 5 --warmup 2 > gpurun_out/r4s_c2ord.log 2>&1
# (then the owner split with its first k entries per thread stored between the rankings: A/B)
cd $GRAFT_REPO_ROOT && for v in own4 own6; do timeout -k 10 400 python -u bench.py --lib tools/abx/libccj_$v.so --sharded --group 32 --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/r4s_sharded_$v.log 2>&1 || exit 1; done && \
timeout -k 10 400 python -u bench.py --sharded --group 32 --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/r4s_sharded_base2.log 2>&1
