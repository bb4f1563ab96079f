set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r5
timeout -k 10 300 python3 -u -m pytest tests/test_probe_gpu.py -x -q -m gpu -k partitioned --timeout 120 --timeout-method thread > gpurun_out/r5/tests.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/r5/tests.log; exit 1; }
tail -3 gpurun_out/r5/tests.log
V="w1_2u_3/1 w1_2u_3 w2_4a_4 w2_4a_4/1 w1_2u_3//16"
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/r5/kt -o kt -- python3 tools/sweep_part.py $V > gpurun_out/r5/kt.log 2>&1 || { echo "kt failed $?"; tail gpurun_out/r5/kt.log; exit 1; }
grep probe gpurun_out/r5/kt.log
python3 tools/trace_split.py gpurun_out/r5/kt $V
