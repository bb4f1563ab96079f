set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r26; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_probe_gpu.py -x -q -m gpu -k "partitioned" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt -o kt -- python3 tools/sweep_part.py w2_4l_3 > $O/c2.log 2>&1 || { echo "c2 failed"; tail $O/c2.log; exit 1; }
grep probe $O/c2.log; python3 tools/trace_split.py $O/kt two512
CCJ_SPLIT_WIDE=1 timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/ktw -o kt -- python3 tools/sweep_part.py w2_4l_3 > $O/c2w.log 2>&1 || { echo "c2w failed"; tail $O/c2w.log; exit 1; }
grep probe $O/c2w.log; python3 tools/trace_split.py $O/ktw one1024
