# GPU box: split tile size sweep (CCJ_SPLIT_PER keys per thread per tile) on the C2 step + parity tests at 13
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r39; mkdir -p $O
for p in ${PERS:-12 13 11 10}; do
  CCJ_SPLIT_PER=$p timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/p$p -o kt -- python3 bench.py --steps 10 --warmup 3 --no-cpu > $O/p$p.json 2> $O/p$p.err || { echo "per $p failed"; tail $O/p$p.err; exit 1; }
  echo "per=$p $(grep -o '"ms_per_step": [0-9.]*' $O/p$p.json) $(grep -o '"l2_ok": [a-z]*' $O/p$p.json | head -1) $(grep -E 'slot_split_fixed|probe_win' $O/p$p/kt_kernel_stats.csv | cut -d, -f1,4 | tr '\n' ' ')"
done
CCJ_SPLIT_PER=13 timeout -k 10 300 python -u -m pytest tests/test_probe_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "partition" > $O/tests13.log 2>&1 || { echo "tests at 13 failed"; tail -20 $O/tests13.log; exit 1; }
tail -1 $O/tests13.log
