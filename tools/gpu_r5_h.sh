# round 5 call H: the walk's pattern without its key loads, and with the keys as 16-byte loads
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
( timeout -k 5 120 ./tools/overlap_emu 256 keys && timeout -k 5 120 ./tools/overlap_emu 256 keys ) > gpurun_out/r5h_walk_keys.log 2>&1
