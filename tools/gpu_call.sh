# round 5 call AI: profiles of C3 (partitioned and reference order) with the spread overflow cursors
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/profile_round.sh r5g c3 c3ord > gpurun_out/r5ai_prof.log 2>&1
