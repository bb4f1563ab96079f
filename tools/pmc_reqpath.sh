#!/bin/bash
# TCP / TA / TD counters of the reqpath microbenchmark (REQPATH_MODE=lanes), to set beside the
# walk's (tools/pmc_ab.sh): requests in flight per CU and L1->L2 latency at the DMA request ceiling.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmc_reqpath
mkdir -p "$OUT"
for grp in "GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  name=$(echo "$grp" | tr ' ' '+')
  REQPATH_MODE=lanes timeout -s KILL 60 rocprofv3 --pmc $grp -T -f csv -d "$OUT/$name" -o pmc -- ./tools/reqpath > "$OUT/$name.log" 2>&1 || { echo "pmc $grp failed rc=$?"; tail -3 "$OUT/$name.log"; exit 1; }
done
echo done
