# GPU box: C5 dense payload (CCJ_PAY_DENSE=1: rows by rank among occupied slots) vs slot-major rows
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r44; mkdir -p $O
CCJ_PAY_DENSE=1 timeout -k 10 300 python -u -m pytest tests/test_c5_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_dense.log 2>&1 || { echo "dense tests failed"; tail -30 $O/tests_dense.log; exit 1; }
tail -1 $O/tests_dense.log
for v in 1 0 1; do
  CCJ_PAY_DENSE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/d$v -o kt -- python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/d$v.json 2> $O/d$v.err || { echo "dense $v failed"; tail $O/d$v.err; exit 1; }
  echo "dense=$v $(grep -o '"ms_per_step": [0-9.]*' $O/d$v.json | head -1) $(grep -o '"[a-z_]*_ok": [a-z]*' $O/d$v.json | tr '\n' ' ') $(grep -E 'gather_payload|slot_split_fixed|probe_win' $O/d$v/kt_kernel_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
done
