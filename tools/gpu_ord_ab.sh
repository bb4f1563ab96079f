#!/bin/bash
# same-box A/B of the ordered (L3) path (tuning build), env strings as arguments; equals_chunk_path_l3 in the log
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/ord_ab.log
for v in "$@"; do
  env $v timeout -k 10 300 python -u bench.py --lib tuning --path ordered --no-cpu --no-verify --steps 8 --warmup 2 > gpurun_out/ord_run.log 2>&1 || { tail -20 gpurun_out/ord_run.log; exit 1; }
  tail -1 gpurun_out/ord_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',round(d['ms_per_step'],3),d['parity'])" >> gpurun_out/ord_ab.log
done
cat gpurun_out/ord_ab.log
