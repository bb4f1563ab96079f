# same-box A/B of the slot walk's row loads: predicated (one wait per load) vs unconditional; twice each
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
P=chunk-compaction-in-vectorized-execution-simd_amd
for v in pred uncond pred uncond; do
  cp $P/libccj_v_$v.so $P/libccj_tuning.so
  CCJ_RANK=0 timeout -k 10 200 python -u bench.py --lib tuning --no-cpu --no-verify --steps 10 > gpurun_out/ab_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',round(d['ms_per_step'],3),[(o['path'],round(o['ms_per_step'],3)) for o in d['other_paths']])" >> gpurun_out/ab_summary.log
done
