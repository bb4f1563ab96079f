# round 4 call V: kernel traces + PMC of c5 and c2ord (tools/profile_round.sh)
cd $GRAFT_REPO_ROOT && bash tools/profile_round.sh r4 c5 c2ord
