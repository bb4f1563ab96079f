set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r7; mkdir -p $O
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -f csv -d $O/kt -o kt -- python3 bench.py --workload c5 --steps 3 --warmup 1 --no-cpu --no-verify > $O/c5p.log 2>&1 || { echo "c5p failed"; tail $O/c5p.log; exit 1; }
head -8 $O/kt/kt_kernel_stats.csv
