# round 4 call P2: final kernel traces + PMC of the C2 and C3 steps (KS = 7 split, chunk-slot walk)
cd $GRAFT_REPO_ROOT && bash tools/profile_round.sh r4 c2 c3
