# round 4 call T: filter walk with non-temporal match stores (nt) against the same tree without (base),
# interleaved twice on one box, C3 stream
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for v in base nt base nt; do timeout -k 10 200 python -u tools/exp_split_c3.py --lib tools/ab/libccj_$v.so c3 > gpurun_out/r4t_$v.log 2>&1 && grep split gpurun_out/r4t_$v.log | sed "s/^/$v /" >> gpurun_out/r4t_all.log || exit 1; done
