# round 4 call W: kernel trace + PMC of c3ord (tools/profile_round.sh)
cd $GRAFT_REPO_ROOT && bash tools/profile_round.sh r4 c3ord
