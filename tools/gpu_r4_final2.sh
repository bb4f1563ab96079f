# round 4 final (second): the whole GPU suite, smoke, the default bench line (C2), and verified C3 and
# C2-ordered lines of the final tree (one-round compaction path, 512-thread unsplit)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4final2_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4final2_smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/r4final2_bench.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu > gpurun_out/r4final2_c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --path ordered --no-cpu --no-other > gpurun_out/r4final2_c2ord.log 2>&1
