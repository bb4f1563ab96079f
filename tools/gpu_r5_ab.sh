# round 5 call AB: multi-GPU and bench tests after the share option, and the one-rank rehearsal line
# with the local probe's full-grid time beside it
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_bench_gpu.py > gpurun_out/r5ab_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --sharded --group 32 --no-cpu > gpurun_out/r5ab_sharded_g32.log 2> gpurun_out/r5ab_sharded_g32.err
