#!/bin/bash
# tools/pmc_walk.sh TAG [bench args] — ON THE GPU BOX: per-unit PMC passes (TA/TD/TCP/TCC busy and
# stall counters) for the C2 walk + split kernels, one counter group per rocprofv3 run.
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmcw_$TAG
mkdir -p "$OUT"
for grp in "GRBM_GUI_ACTIVE GRBM_COUNT" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCC_BUSY_sum TCC_TAG_STALL_sum TCC_READ_SECTORS_sum TCC_EA0_RDREQ_LEVEL_sum" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
           "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  name=$(echo "$grp" | tr ' ' '+')
  echo "[pmc] $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_KERNEL:-slot_split|probe_walk}" -T -f csv -d "$OUT/$name" -o pmc \
      -- python3 bench.py "$@" --steps 2 --warmup 1 --no-cpu --no-verify --no-other > "$OUT/$name.log" 2>&1 || { echo "pmc $grp failed rc=$?"; tail -3 "$OUT/$name.log"; }
done
echo "[pmc] done"
