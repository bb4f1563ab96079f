set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r22; mkdir -p $O
V="w2_4u_3 w2_4l_3 w2_4s_3"
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt -o kt -- python3 tools/sweep_part.py $V > $O/c2.log 2>&1 || { echo "c2 failed"; tail $O/c2.log; exit 1; }
grep probe $O/c2.log
python3 tools/trace_split.py $O/kt $V
