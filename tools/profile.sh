#!/bin/bash
# tools/profile.sh TAG [bench args...] — run ON THE GPU BOX (via gpurun).
# 1) kernel trace + stats of the bench command; 2) PMC passes, one counter group per run (FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950: MI355X_MICROARCH.md §rocprofv3 PMC slots).
# Outputs under gpurun_out/prof_TAG/; tools/prof_summary.py turns them into profiles/ files.
set -o pipefail
TAG=$1; shift
ARGS="$@"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
# the build the counters belong to (ccj_build_hash; bench.py refuses the traffic of another build)
python3 -c "import sys; sys.path.insert(0, 'chunk-compaction-in-vectorized-execution-simd_amd'); import ccj; print(ccj.build_hash())" > "$OUT/build_hash.txt" || exit 1
echo "[profile] kernel trace: bench.py $ARGS"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/kt" -o kt -- python3 bench.py $ARGS > "$OUT/kt_bench.log" 2>&1 || exit $?
for grp in FETCH_SIZE WRITE_SIZE "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE"; do
  name=$(echo "$grp" | tr ' ' '+')
  echo "[profile] pmc $grp"
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_KERNEL:-slot_split_fixed|probe_walk}" -T -f csv -d "$OUT/pmc_$name" -o pmc \
      -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu --no-verify > "$OUT/pmc_$name.log" 2>&1 || { echo "pmc $grp failed rc=$?"; tail -5 "$OUT/pmc_$name.log"; }
done
echo "[profile] done"
