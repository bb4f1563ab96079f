# round 4 call Q: C3 split + filter walk at chain window bits 18 (default) and 17 (CCJ_WINDOW_BITS=18,
# tuning build), interleaved twice on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 200 python -u tools/exp_split_c3.py --lib tuning c3 c3h0 > gpurun_out/r4q_wb18a.log 2>&1 && \
CCJ_WINDOW_BITS=18 timeout -k 10 200 python -u tools/exp_split_c3.py --lib tuning c3 c3h0 > gpurun_out/r4q_wb17a.log 2>&1 && \
timeout -k 10 200 python -u tools/exp_split_c3.py --lib tuning c3 c3h0 > gpurun_out/r4q_wb18b.log 2>&1 && \
CCJ_WINDOW_BITS=18 timeout -k 10 200 python -u tools/exp_split_c3.py --lib tuning c3 c3h0 > gpurun_out/r4q_wb17b.log 2>&1
