# round 5 call BF: per-unit counters of the final C5 gather (gather_payload_cols) — which unit holds it now
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
PMC_KERNEL="gather_payload_cols" bash tools/unit_pass.sh r5u3_c5 --workload c5 > gpurun_out/r5bf_c5.log 2>&1
