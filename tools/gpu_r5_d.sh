# round 5 call D: C3 filter-walk ablations (records / chains from a half or a quarter of the
# partition's buckets; L2-resident keys) to size the walk's L2 working-set cost, then kernel
# traces + counter passes of C5 and the two reference-order paths with the current kernels
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/gpu_ab.sh r5abl c3split 2 tuning tuning:CCJ_ABLATE=16384 tuning:CCJ_ABLATE=32768 tuning:CCJ_ABLATE=65536 tuning:CCJ_ABLATE=98304 > gpurun_out/r5abl_ab.log 2>&1 && \
timeout -k 10 1000 bash tools/profile_round.sh r5 c5 c2ord c3ord > gpurun_out/r5d_prof.log 2>&1
