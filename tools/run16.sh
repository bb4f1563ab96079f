set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r16; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_probe_gpu.py tests/test_dist_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python3 bench.py --sharded --steps 3 --warmup 1 --no-cpu > $O/sharded.json 2> $O/sharded.err || { echo "sharded failed"; tail $O/sharded.err; exit 1; }
cat $O/sharded.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o kt -- python3 tools/sweep_part.py w2_4a_4 > $O/c2.log 2>&1 || { echo "c2 failed"; exit 1; }
grep probe $O/c2.log; grep -E "slot_split|probe_win" $O/kt/kt_kernel_stats.csv
