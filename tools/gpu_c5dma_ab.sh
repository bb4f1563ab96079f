#!/bin/bash
# same-box A/B of the C5 payload gather (tuning build): CCJ_GATHER_DMA 0 = gather_payload_quad
# (vector loads), 1 / 2 = gather_payload_dma<4 / 8> (LDS-DMA row pieces); payload_cols_ok in the log
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/c5dma_ab.log
for v in "$@"; do
  env $v timeout -k 10 300 python -u bench.py --lib tuning --workload c5 --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/c5dma_run.log 2>&1 || { tail -20 gpurun_out/c5dma_run.log; exit 1; }
  tail -1 gpurun_out/c5dma_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',round(d['ms_per_step'],3),d['parity'])" >> gpurun_out/c5dma_ab.log
done
cat gpurun_out/c5dma_ab.log
