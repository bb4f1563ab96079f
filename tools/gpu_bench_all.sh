#!/bin/bash
# every workload's bench line on one box (round summary): gpurun_out/bench_all.log
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/bench_all.log
run() {
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench_all_run.log 2>&1 || { tail -20 gpurun_out/bench_all_run.log; exit 1; }
  tail -1 gpurun_out/bench_all_run.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());r=d.get('roofline') or {}
print('$*', '|', round(d['ms_per_step'],3), 'ms |', round(d['value']/1e9,2), 'G/s | frac', r.get('frac') and round(r['frac'],4), '|', {k:v for k,v in d['parity'].items() if k in ('l1_ok','l2_ok','payload_cols_ok','equals_chunk_path_l3','compaction_keeps_all','modes_agree')})" >> gpurun_out/bench_all.log
}
run --no-cpu --no-other
run --no-cpu --no-other --path ordered
run --no-cpu --no-other --path chunk
run --no-cpu --workload c3
run --no-cpu --workload c3 --path ordered
run --no-cpu --workload c5
run --no-cpu --workload pipeline
run --gpus 1 --sharded --no-cpu --steps 5 --warmup 2
cat gpurun_out/bench_all.log
