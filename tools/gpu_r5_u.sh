# round 5 call U: final-tree profiles of the C2 and C3 steps (kernel trace + HBM counters) and the
# per-unit counter passes of the C2 kernels
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/profile_round.sh r5f c2 c3 > gpurun_out/r5u_prof.log 2>&1 && \
PMC_KERNEL="slot_split_pipe|probe_walk2" bash tools/unit_pass.sh r5u2_c2 --no-other --no-other-workloads > gpurun_out/r5u_units.log 2>&1
