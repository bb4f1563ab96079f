# round 5 call S: per-unit counter passes over the C2 headline's two kernels (split, walk)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
PMC_KERNEL="slot_split_pipe|probe_walk2" bash tools/unit_pass.sh r5u_c2 --no-other --no-other-workloads
