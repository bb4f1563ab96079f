# round 5 call C: the default bench line (C2 + other paths + C3/C5), then kernel traces + counter
# passes of C2 and C3 with the current kernels, and the split's store+read floor on the same box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u bench.py > gpurun_out/r5c_bench.log 2> gpurun_out/r5c_bench.err && \
( for a in "22 1 read 512 8" "22 1 both 512 8"; do timeout -k 5 60 ./tools/runstore $a || exit 1; done ) > gpurun_out/r5c_runstore.log 2>&1 && \
timeout -k 10 900 bash tools/profile_round.sh r5 c2 c3 > gpurun_out/r5c_prof.log 2>&1
