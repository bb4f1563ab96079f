# round 4 call R: deferred overflow replies in the split — same-box A/B against the round-start build
# (tools/ab/libccj_head.so), interleaved twice: C3 streams and the C2 line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 200 python -u tools/exp_split_c3.py --lib tools/ab/libccj_head.so c3 c3h0 > gpurun_out/r4r_head_a.log 2>&1 && \
timeout -k 10 200 python -u tools/exp_split_c3.py c3 c3h0 > gpurun_out/r4r_new_a.log 2>&1 && \
timeout -k 10 200 python -u tools/exp_split_c3.py --lib tools/ab/libccj_head.so c3 c3h0 > gpurun_out/r4r_head_b.log 2>&1 && \
timeout -k 10 200 python -u tools/exp_split_c3.py c3 c3h0 > gpurun_out/r4r_new_b.log 2>&1 && \
timeout -k 10 150 python -u bench.py --lib tools/ab/libccj_head.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4r_c2_head.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4r_c2_new.log 2>&1 && \
timeout -k 10 150 python -u bench.py --lib tools/ab/libccj_head.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4r_c2_head2.log 2>&1 && \
timeout -k 10 150 python -u bench.py --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4r_c2_new2.log 2>&1
