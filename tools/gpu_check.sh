# the round-end checks: GPU suite, smoke, the default bench line, a kernel trace of the ordered path
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/kt_ord -o kt -- python3 bench.py --path ordered --no-other --no-cpu --no-verify --steps 5 > gpurun_out/kt_ord.log 2>&1
