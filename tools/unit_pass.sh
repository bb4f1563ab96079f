#!/bin/bash
# tools/unit_pass.sh TAG [bench args...] — ON THE GPU BOX: per-unit PMC passes over one bench.py
# command (which unit of the CU's memory pipeline holds each kernel: TA / TD / TCP busy and stall
# cycles, SQ issue and wait cycles, LDS bank conflicts).  One counter group per run, within the
# gfx950 per-pass slots (TA 2, TD 2, TCP 4, SQ 8, GRBM 2); tools/unit_summary.py TAG turns the
# output into profiles/TAG_units.json.
set -o pipefail
TAG=$1; shift
ARGS="$@"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
for grp in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_WAVEFRONTS_sum GRBM_GUI_ACTIVE" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE"; do
  name=$(echo "$grp" | tr ' ' '+')
  echo "[units] pmc $grp"
  timeout -s KILL 180 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_KERNEL:-slot_split_pipe|probe_walk}" -T -f csv -d "$OUT/pmc_$name" -o pmc \
      -- python3 bench.py $ARGS --steps 2 --warmup 1 --no-cpu --no-verify > "$OUT/pmc_$name.log" 2>&1 || { echo "pmc $grp failed rc=$?"; tail -5 "$OUT/pmc_$name.log"; exit 1; }
done
echo "[units] done"
