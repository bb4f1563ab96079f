# same-box A/B of the ordered path: previous kernels (v_old) against the new (v_new), three times
# each; first the ordered-path parity tests on the new product library
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/loads_ab.log
timeout -k 10 300 python -u -m pytest tests/test_probe_gpu.py -k ordered -x -q --timeout 200 --timeout-method thread > gpurun_out/ord_tests.log 2>&1 || exit 1
P=chunk-compaction-in-vectorized-execution-simd_amd
for v in old new old new old new; do
  cp $P/libccj_v_$v.so $P/libccj_tuning.so
  timeout -k 10 200 python -u bench.py --lib tuning --no-cpu --steps 10 --path ordered --no-other > gpurun_out/lab.log 2>&1 || exit 1
  tail -1 gpurun_out/lab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',round(d['ms_per_step'],3),d['parity'].get('l1_ok'),d['parity'].get('l2_ok'))" >> gpurun_out/loads_ab.log
done
