# chunk path (probe_chunks) emit staged in LDS: its parity tests (probe, facade, pipelines) on the
# product library, then a same-box A/B of the C2 chunk path (v_old against v_new), three times each
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/chunk_ab.log
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_facade_gpu.py tests/test_pipeline_gpu.py tests/test_pipeline_device_gpu.py tests/test_compact_gpu.py tests/test_c3_gpu.py tests/test_c5_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/chunk_tests.log 2>&1 || exit 1
P=chunk-compaction-in-vectorized-execution-simd_amd
for v in old new old new old new; do
  cp $P/libccj_v_$v.so $P/libccj_tuning.so
  timeout -k 10 200 python -u bench.py --lib tuning --no-cpu --steps 5 --path chunk --no-other > gpurun_out/lab.log 2>&1 || exit 1
  tail -1 gpurun_out/lab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v',round(d['ms_per_step'],3),d['parity'].get('l1_ok'),d['parity'].get('l2_ok'))" >> gpurun_out/chunk_ab.log
done
