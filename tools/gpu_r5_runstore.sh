# round 5: the split's store phase by run length, alignment, partitions and tile groups
# (tools/runstore.hip), and scalar-path L2 reads beside the vector L1 (tools/sreq.hip)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && (
for L in 8 11 16 22 32 44 64; do timeout -k 5 60 ./tools/runstore $L 0 both || exit 1; done
for L in 16 22 32; do timeout -k 5 60 ./tools/runstore $L 1 both || exit 1; done
for L in 16 22; do for w in keys rows; do timeout -k 5 60 ./tools/runstore $L 1 $w || exit 1; done; done
for pg in "22 512 1" "22 64 8" "22 64 1" "176 64 8" "44 256 8" "88 128 8" "11 1024 8" "11 1024 1"; do
  set -- $pg; timeout -k 5 60 ./tools/runstore $1 1 both $2 $3 || exit 1; done
timeout -k 5 60 ./tools/copybench || true
) > gpurun_out/r5_runstore.log 2>&1
( for m in "vec 0" "sca 8" "mix 8" "mix 16" "mix 32"; do timeout -k 5 60 ./tools/sreq $m || exit 1; done ) > gpurun_out/r5_sreq.log 2>&1
