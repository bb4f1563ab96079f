cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && (
for L in 8 11 16 22 32 44 64; do timeout -k 5 60 ./tools/runstore $L 0 both || exit 1; done
for L in 16 22 32; do timeout -k 5 60 ./tools/runstore $L 1 both || exit 1; done
for L in 16 22; do for w in keys rows; do timeout -k 5 60 ./tools/runstore $L 0 $w || exit 1; timeout -k 5 60 ./tools/runstore $L 1 $w || exit 1; done; done
timeout -k 5 60 ./tools/copybench || true
) > gpurun_out/r5_runstore.log 2>&1
