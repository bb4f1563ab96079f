# round 4 call L: the C3 table's split under three probe streams (skewed / unskewed / all hits), and
# the tuning build's no-store ablation of the same
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 240 python -u tools/exp_split_c3.py > gpurun_out/r4l_split.log 2>&1 && \
CCJ_ABLATE=16 timeout -k 10 240 python -u tools/exp_split_c3.py --lib tuning c3 c3h0 > gpurun_out/r4l_split_nostore.log 2>&1
