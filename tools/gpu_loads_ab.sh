# same-box A/B of the unserialized loads (emit_ordered, unsplit_words, gather_payload_quad,
# probe_chain_win): the previous kernels (v_old) against the new (v_new), twice each
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/loads_ab.log
P=chunk-compaction-in-vectorized-execution-simd_amd
for v in old new old new; do
  cp $P/libccj_v_$v.so $P/libccj_tuning.so
  for w in "--path ordered --no-other" "--workload c3" "--workload c5"; do
    timeout -k 10 200 python -u bench.py --lib tuning --no-cpu --steps 5 $w > gpurun_out/lab.log 2>&1 || exit 1
    tail -1 gpurun_out/lab.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v','$w',round(d['ms_per_step'],3),d['parity'].get('l1_ok'),d['parity'].get('l2_ok'),d['parity'].get('payload_cols_ok'),d['parity'].get('compaction_keeps_all'),d['parity'].get('equals_chunk_path_l3'))" >> gpurun_out/loads_ab.log
  done
done
