# round 5 call F: can the walk's L2-request-bound work and the split's HBM-bound stores share the
# chip?  LDS-light emulations of both, alone and together (tools/overlap_emu.hip)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
( for w in 256 128 64; do timeout -k 5 120 ./tools/overlap_emu $w || exit 1; done ) > gpurun_out/r5f_overlap.log 2>&1
