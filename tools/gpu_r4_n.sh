# round 4 call N: same-box A/B of the split (HEAD build vs the working tree) under the C3 streams,
# and the C2 bench line of both
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 240 python -u tools/exp_split_c3.py --lib tools/ab/libccj_head.so c3 c3h0 > gpurun_out/r4n_split_head.log 2>&1 && \
timeout -k 10 240 python -u tools/exp_split_c3.py c3 c3h0 > gpurun_out/r4n_split_new.log 2>&1 && \
timeout -k 10 240 python -u tools/exp_split_c3.py --lib tools/ab/libccj_head.so c3 c3h0 > gpurun_out/r4n_split_head2.log 2>&1 && \
timeout -k 10 150 python -u bench.py --lib tools/ab/libccj_head.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4n_c2_head.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4n_c2_new.log 2>&1
