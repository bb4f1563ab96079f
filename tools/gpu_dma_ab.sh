#!/bin/bash
# same-box A/B of the walk (tuning build): CCJ_WALK_DMA 0 = probe_walk (lane pairs, vector loads),
# 1 = probe_walk with LDS-DMA windows, 2 = probe_walk1 (one lane per row, LDS-DMA ring of
# CCJ_WALK_NB batches); parity of every run in the log
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/dma_ab.log
run() {
  env "$@" timeout -k 10 200 python -u bench.py --lib tuning --no-other --no-cpu --no-verify --steps 10 > gpurun_out/dma_ab_run.log 2>&1 || { tail -20 gpurun_out/dma_ab_run.log; exit 1; }
  tail -1 gpurun_out/dma_ab_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$*',round(d['ms_per_step'],3),d['roofline']['kernel_ms'],d['parity'])" >> gpurun_out/dma_ab.log
}
for v in "$@"; do run $v || exit 1; done
cat gpurun_out/dma_ab.log
