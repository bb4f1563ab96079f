#!/bin/bash
# same-box A/B of the C3 workload (tuning build), env strings as arguments; parity in the log
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/c3_ab.log
for v in "$@"; do
  env $v timeout -k 10 300 python -u bench.py --lib tuning --workload c3 --no-cpu --no-verify --steps 5 --warmup 2 > gpurun_out/c3_run.log 2>&1 || { tail -20 gpurun_out/c3_run.log; exit 1; }
  tail -1 gpurun_out/c3_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',round(d['ms_per_step'],3),'probe',round(d['roofline']['kernel_ms'],3),'comp',round(d['compaction_ms'],3),d['parity'])" >> gpurun_out/c3_ab.log
done
cat gpurun_out/c3_ab.log
