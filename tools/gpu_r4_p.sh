# round 4 call P: kernel traces + PMC passes of the C3 and C2 steps (tools/profile_round.sh)
cd $GRAFT_REPO_ROOT && bash tools/profile_round.sh r4 c3 c2
