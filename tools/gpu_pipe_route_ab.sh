#!/bin/bash
# same-box A/B of ccj_pipeline_run's probe route at large table sizes (tuning build for both arms):
# CCJ_PIPE_ORDERED=1 (tables >= 2^22 slots / buckets through ccj_probe_ordered) vs 0 (probe_chunks).
# tools/gpu_pipe_route_ab.sh LHS RHS  -> gpurun_out/pipe_route_ab.log
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out /tmp/tlib && rm -f gpurun_out/pipe_route_ab.log
ln -sf "$PWD/chunk-compaction-in-vectorized-execution-simd_amd/libccj_tuning.so" /tmp/tlib/libccj.so
LHS=${1:-33554432}; RHS=${2:-33554432}
for table in chain lp; do
  for o in 1 0; do
    CCJ_PIPE_ORDERED=$o LD_LIBRARY_PATH=/tmp/tlib:$LD_LIBRARY_PATH timeout -k 10 400 python -u bench.py --workload pipeline \
      --pipe-table $table --pipe-lhs $LHS --pipe-rhs $RHS --pipe-block 2048 --steps 3 --warmup 1 --no-cpu \
      > gpurun_out/pipe_route_run.log 2>&1 || { tail -20 gpurun_out/pipe_route_run.log; exit 1; }
    tail -1 gpurun_out/pipe_route_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$table ordered=$o','full',round(d['ms_per_step'],2),'none',round(d['no_compaction']['ms_per_step'],2),'dyn',round(d['dynamic_compaction']['ms_per_step'],2),d['parity'])" >> gpurun_out/pipe_route_ab.log
  done
done
cat gpurun_out/pipe_route_ab.log
