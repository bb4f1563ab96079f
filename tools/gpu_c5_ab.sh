# C5 walk with positions (probe_walk<..., POS>) vs probe_win: parity tests on the product library, then
# a same-box A/B of the C5 bench (previous kernels v_old against v_new), three times each
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/c5_ab.log
timeout -k 10 400 python -u -m pytest tests/test_c5_gpu.py tests/test_probe_gpu.py -k "c5 or partitioned or walks" -x -q --timeout 200 --timeout-method thread > gpurun_out/c5_tests.log 2>&1 || exit 1
P=chunk-compaction-in-vectorized-execution-simd_amd
for v in old new old new old new; do
  cp $P/libccj_v_$v.so $P/libccj_tuning.so
  timeout -k 10 200 python -u bench.py --lib tuning --no-cpu --steps 5 --workload c5 > gpurun_out/lab.log 2>&1 || exit 1
  tail -1 gpurun_out/lab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',round(d['ms_per_step'],3),d['parity'].get('l1_ok'),d['parity'].get('l2_ok'),d['parity'].get('payload_cols_ok'))" >> gpurun_out/c5_ab.log
done
