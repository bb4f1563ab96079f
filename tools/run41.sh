# GPU box: split variant keeping each image row's partition in LDS (CCJ_SPLIT_SD=1, 9/10 keys per thread) vs the default
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r41; mkdir -p $O
for v in "11 0" "10 1" "9 1" "11 0" "10 1"; do
  set -- $v
  CCJ_SPLIT_PER=$1 CCJ_SPLIT_SD=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/p$1s$2 -o kt -- python3 bench.py --steps 10 --warmup 3 --no-cpu > $O/p$1s$2.json 2> $O/p$1s$2.err || { echo "per $1 sd $2 failed"; tail $O/p$1s$2.err; exit 1; }
  echo "per=$1 sd=$2 $(grep -o '"ms_per_step": [0-9.]*' $O/p$1s$2.json | head -1) $(grep -o '"l2_ok": [a-z]*' $O/p$1s$2.json | head -1) $(grep -E 'slot_split_fixed|probe_win' $O/p$1s$2/kt_kernel_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
done
CCJ_SPLIT_PER=10 CCJ_SPLIT_SD=1 timeout -k 10 300 python -u -m pytest tests/test_probe_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "partition or shard" > $O/tests_sd.log 2>&1 || { echo "tests sd failed"; tail -20 $O/tests_sd.log; exit 1; }
tail -1 $O/tests_sd.log
