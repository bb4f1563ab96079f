# round 5 call V: final-tree profiles of C5 and both reference-order paths
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/profile_round.sh r5f c5 c2ord c3ord > gpurun_out/r5v_prof.log 2>&1
