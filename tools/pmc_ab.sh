#!/bin/bash
# tools/pmc_ab.sh TAG KERNEL_REGEX "ENV1" "ENV2" ... -- bench args   (ON THE GPU BOX)
# Unit / instruction-mix PMC passes of one kernel for several tuning-build variants (one env string
# per variant), one counter group per rocprofv3 run; tools/pmc_ab_summary.py prints the table.
TAG=$1; RE=$2; shift 2
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ "$1" == "--" ] && shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmcab_$TAG
mkdir -p "$OUT"
for vi in "${!VARS[@]}"; do
  v="${VARS[$vi]}"
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
             "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
             "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
             "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA" \
             "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INSTS_LDS_LOAD"; do
    name=$(echo "$grp" | tr ' ' '+')
    d="$OUT/v$vi/$name"
    mkdir -p "$d"
    echo "$v" > "$OUT/v$vi/env"
    env $v timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -T -f csv -d "$d" -o pmc \
        -- python3 bench.py --lib tuning "$@" --steps 2 --warmup 1 --no-cpu --no-verify --no-other > "$d.log" 2>&1 || { echo "pmc $v / $grp failed rc=$?"; tail -3 "$d.log"; }
  done
done
echo "[pmc_ab] done"
