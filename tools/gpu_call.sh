# round 5 call BE: the C2 headline profile (kernel trace + counters) of the final tree
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/profile_round.sh r5k c2 > gpurun_out/r5be_prof.log 2>&1
