set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r30; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -T -f csv -d $O/kt -o kt -- python3 tools/overlap_part.py 1/1 2/1 2/2 4/1 4/2 8/2 > $O/ov.log 2>&1 || { echo "ov failed"; tail $O/ov.log; exit 1; }
cat $O/ov.log
