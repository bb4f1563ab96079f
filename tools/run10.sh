set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r10; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_probe_gpu.py tests/test_c5_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt3 -o kt -- python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu > $O/c3p.json 2> $O/c3p.err || { echo "c3p failed"; tail $O/c3p.err; exit 1; }
cat $O/c3p.json
head -8 $O/kt3/kt_kernel_stats.csv
timeout -k 10 300 python3 tools/sweep_part.py w2_4a_4 w2_4a_4 > $O/c2.log 2>&1 || { echo "c2 failed"; tail $O/c2.log; exit 1; }
cat $O/c2.log
