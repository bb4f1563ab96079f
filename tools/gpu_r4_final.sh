# round 4 final: the whole GPU suite, smoke, and the default bench line (C2) of the committed tree
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4final_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4final_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r4final_bench.log 2>&1
