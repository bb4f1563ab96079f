set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r28; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt -o kt -- python3 tools/sweep_part.py w2_4l_3 w2_4l_3q > $O/c2.log 2>&1 || { echo "c2 failed"; tail $O/c2.log; exit 1; }
grep probe $O/c2.log; python3 tools/trace_split.py $O/kt w2_4l_3 w2_4l_3q
for Q in 4 5 8; do
CCJ_PROBE_QUEUE=$Q timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt$Q -o kt -- python3 tools/sweep_part.py w2_4l_3q > $O/c2_$Q.log 2>&1 || { echo "c2 $Q failed"; tail $O/c2_$Q.log; exit 1; }
grep probe $O/c2_$Q.log | cut -c1-200; python3 tools/trace_split.py $O/kt$Q q$Q
done
