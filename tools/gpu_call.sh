# round 5 call BH: round-end checks on the final tree — the whole GPU suite, smoke, and the driver's
# bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5bh_gputest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5bh_smoke.log 2>&1 && \
timeout -k 10 500 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5bh_bench.log 2> gpurun_out/r5bh_bench.err
