# round 5 call G: the split's store pattern with the split's own load schedule (next tile's keys in
# flight during this tile's stores) against the plain forms, and the product C2 split, same box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
( for a in "22 1 pref 512 8" "22 1 read 512 8" "22 1 both 512 8" "44 1 pref 256 8" "22 1 pref 512 8"; do
    timeout -k 5 60 ./tools/runstore $a || exit 1; done ) > gpurun_out/r5g_runstore.log 2>&1 && \
timeout -k 10 200 python -u bench.py --no-cpu --no-other --no-other-workloads --no-verify --steps 10 --warmup 3 > gpurun_out/r5g_c2.log 2>&1
