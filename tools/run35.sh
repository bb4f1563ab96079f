# GPU box: C5 gather variants (CCJ_GATHER_VARIANT = U*100 + plain_stores*10 + xcd_swizzle)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r35; mkdir -p $O
for v in 400 200 800 410 401 411 801; do
  CCJ_GATHER_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/g$v -o kt -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > $O/g$v.json 2> $O/g$v.err || { echo "variant $v failed"; tail $O/g$v.err; exit 1; }
  echo "$v $(grep -o '"payload_cols_ok": [a-z]*' $O/g$v.json) $(grep gather_payload $O/g$v/kt_kernel_stats.csv | cut -d, -f1,4)"
done
