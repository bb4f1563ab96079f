# GPU box: table window size x split tile size with the walk of r1h (CCJ_WINDOW_BITS 18/19/20, CCJ_SPLIT_PER)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r43; mkdir -p $O
for v in "19 11" "18 11" "18 12" "18 10" "20 11" "20 13" "19 11"; do
  set -- $v
  CCJ_WINDOW_BITS=$1 CCJ_SPLIT_PER=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/w$1p$2 -o kt -- python3 bench.py --steps 10 --warmup 3 --no-cpu > $O/w$1p$2.json 2> $O/w$1p$2.err || { echo "w $1 p $2 failed"; tail $O/w$1p$2.err; exit 1; }
  echo "w=$1 per=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/w$1p$2.json | head -1) $(grep -o '"l2_ok": [a-z]*' $O/w$1p$2.json | head -1) $(grep -E 'slot_split_fixed|probe_win' $O/w$1p$2/kt_kernel_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
done
