# round 5 call E: the whole GPU suite and the smoke on the current tree, then the one-rank
# rehearsal of the N > 1 step (own segment copied locally now, no RCCL self-copy), groups of 32
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5e_tests.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5e_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --sharded --group 32 --no-cpu > gpurun_out/r5e_sharded_g32.log 2> gpurun_out/r5e_sharded_g32.err
