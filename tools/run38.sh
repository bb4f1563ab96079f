# GPU box: split/walk overlap across streams (tools/overlap_part.py pieces/streams)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r38; mkdir -p $O
timeout -k 10 500 python3 -u tools/overlap_part.py 1/1 2/1 2/2 4/1 4/2 8/2 8/4 > $O/overlap.log 2>&1 || { echo "overlap failed"; tail -20 $O/overlap.log; exit 1; }
cat $O/overlap.log
