set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r18; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_dist_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V="w2_4a_4 w2_4a_4//512"
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt -o kt -- python3 tools/sweep_part.py $V > $O/c2.log 2>&1 || { echo "c2 failed"; exit 1; }
grep probe $O/c2.log
python3 tools/trace_split.py $O/kt $V
