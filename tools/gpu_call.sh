# round 5 call AX: the C5 profile (kernel trace + counters) of the final tree's five-workgroup gather
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/profile_round.sh r5i c5 > gpurun_out/r5ax_prof.log 2>&1
