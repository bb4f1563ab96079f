# round 5 call AN: HBM write-only / read-only / copy rates at C5's column sizes (tools/write_bw.py)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u tools/write_bw.py > gpurun_out/r5an_write_bw.log 2>&1
