# round 5 call Z: per-unit counter passes over the other workloads' kernels (C3 split + filter walk,
# C5 walk + gather, the ordered route's walk, unsplit and emit)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
PMC_KERNEL="slot_split_pipe|probe_chain_filt" bash tools/unit_pass.sh r5u_c3 --workload c3 > gpurun_out/r5z_c3.log 2>&1 && \
PMC_KERNEL="probe_walk2|gather_payload_quad" bash tools/unit_pass.sh r5u_c5 --workload c5 > gpurun_out/r5z_c5.log 2>&1 && \
PMC_KERNEL="probe_walk1|unsplit_words|emit_ordered" bash tools/unit_pass.sh r5u_c2ord --path ordered --no-other --no-other-workloads > gpurun_out/r5z_c2ord.log 2>&1
