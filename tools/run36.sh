# GPU box: PMC counters of the C5 payload gather (and its walk) — what bounds gather_payload_quad
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
PMC_KERNEL='gather_payload_quad|probe_win' timeout -k 10 900 bash tools/profile.sh r1g_c5 --workload c5 --steps 2 --warmup 1 --no-cpu > gpurun_out/r36.log 2>&1 || { echo "profile failed"; tail gpurun_out/r36.log; exit 1; }
tail -3 gpurun_out/r36.log
