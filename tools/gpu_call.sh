# round 5 call AH: the slot split's segment cursors 1 / 4 / 8 u32 apart within an XCD group
# (32 / 8 / 4 per 128-byte line) — C2 and C3, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5sp c2 2 product tools/abx/libccj_sp4.so tools/abx/libccj_sp8.so > gpurun_out/r5sp_ab.log 2>&1 && \
bash tools/gpu_ab.sh r5sp3 c3 2 product tools/abx/libccj_sp4.so tools/abx/libccj_sp8.so > gpurun_out/r5sp3_ab.log 2>&1
