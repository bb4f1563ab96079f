set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r8; mkdir -p $O
timeout -k 10 600 python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/c5p.json 2> $O/c5p.err || { echo "c5p failed"; tail $O/c5p.err; exit 1; }
cat $O/c5p.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o kt -- python3 bench.py --workload c5 --path chunk --steps 5 --warmup 2 --no-cpu > $O/c5c.json 2> $O/c5c.err || { echo "c5c failed"; tail $O/c5c.err; exit 1; }
cat $O/c5c.json
head -6 $O/kt/kt_kernel_stats.csv
