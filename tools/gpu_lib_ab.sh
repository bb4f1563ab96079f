#!/bin/bash
# same-box A/B of two library builds: tools/gpu_lib_ab.sh WORKLOAD_ARGS LIB1 LIB2 ... (each LIB a
# .so path or "tuning"); every run's ms/step and parity in gpurun_out/lib_ab.log
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/lib_ab.log
ARGS=$1; shift
for lib in "$@"; do
  timeout -k 10 300 python -u bench.py --lib $lib $ARGS --no-cpu --no-verify --no-other --steps 8 --warmup 2 > gpurun_out/lib_run.log 2>&1 || { tail -20 gpurun_out/lib_run.log; exit 1; }
  tail -1 gpurun_out/lib_run.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$lib $ARGS',round(d['ms_per_step'],3),d['roofline']['kernel_ms'],d['parity'])" >> gpurun_out/lib_ab.log
done
cat gpurun_out/lib_ab.log
