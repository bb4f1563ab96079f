set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r12; mkdir -p $O
for G in 0 6 12 24; do
  CCJ_PROBE_GRID=$G timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt$G -o kt -- python3 tools/sweep_part.py w2_4a_4 > $O/c2_$G.log 2>&1 || { echo "c2 $G failed"; tail $O/c2_$G.log; exit 1; }
  grep probe $O/c2_$G.log
  python3 tools/trace_split.py $O/kt$G "grid$G"
done
