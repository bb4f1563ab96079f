set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r33; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_probe_gpu.py tests/test_c5_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt -o kt -- python3 tools/sweep_part.py w2_4l_3 w2_4u_3 > $O/c2.log 2>&1 || { echo "c2 failed"; tail $O/c2.log; exit 1; }
grep probe $O/c2.log | cut -c1-200; python3 tools/trace_split.py $O/kt w2_4l_3 w2_4u_3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $O/c5 -o kt -- python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; tail $O/c5.err; exit 1; }
cut -c1-400 $O/c5.json; head -6 $O/c5/kt_kernel_stats.csv | cut -c1-150
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $O/c3 -o kt -- python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu > $O/c3.json 2> $O/c3.err || { echo "c3 failed"; tail $O/c3.err; exit 1; }
cut -c1-400 $O/c3.json; head -8 $O/c3/kt_kernel_stats.csv | cut -c1-150
