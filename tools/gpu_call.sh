# round 5 call AG: each tile group's segment cursors on their own 128-byte line (few partitions) —
# multi-GPU / partitioned tests, the owner split alone against the packed build, the rehearsal line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dist_gpu.py tests/test_probe_gpu.py -k "dist or partition or sharded or owner or grouped or segment" > gpurun_out/r5ag_tests.log 2>&1 && \
o=gpurun_out/r5ag_owner.log && : > $o && \
for i in 1 2; do
  echo "== product $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --unmasked >> $o 2>&1 && \
  echo "== packed $i" >> $o && timeout -k 10 120 python3 -u tools/owner_split_bench.py --lib tools/abx/libccj_packed.so --unmasked >> $o 2>&1 || exit 1
done && \
timeout -k 10 300 python -u bench.py --gpus 1 --sharded --group 32 --no-cpu > gpurun_out/r5ag_sharded_g32.log 2> gpurun_out/r5ag_sharded_g32.err
