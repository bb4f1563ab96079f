# GPU box: split ablations (per-kernel times from a kernel trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r3
V="w1_2u_3/3 w1_2u_3/3/16 w1_2u_3/3/32 w1_2u_3/3/64 w1_2u_3/3/48 w1_2u_3/3/112 w1_2u_3/1 w2_4a_4/3"
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/r3/kt -o kt -- python3 tools/sweep_part.py $V > gpurun_out/r3/kt.log 2>&1 || { echo "kt failed $?"; tail gpurun_out/r3/kt.log; exit 1; }
grep probe gpurun_out/r3/kt.log
python3 tools/trace_split.py gpurun_out/r3/kt $V
