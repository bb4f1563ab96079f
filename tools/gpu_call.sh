# round 5 call BC: the C5 profile (kernel trace + counters) of the final tree (per-lane position loads)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/profile_round.sh r5j c5 > gpurun_out/r5bc_prof.log 2>&1
