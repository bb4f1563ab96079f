set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r4
V="w1_2u_3/3 w1_2u_3/1 w1_2u_3/3/128 w1_2u_3/3/256 w1_2u_3/3/16"
timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/r4/kt -o kt -- python3 tools/sweep_part.py $V > gpurun_out/r4/kt.log 2>&1 || { echo "kt failed $?"; tail gpurun_out/r4/kt.log; exit 1; }
python3 tools/trace_split.py gpurun_out/r4/kt $V
V2="w1_2u_3/3 w1_2u_3/1 w2_4a_4/1"
CCJ_WINDOW_BITS=19 timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/r4/kt19 -o kt -- python3 tools/sweep_part.py $V2 > gpurun_out/r4/kt19.log 2>&1 || { echo "kt19 failed $?"; tail gpurun_out/r4/kt19.log; exit 1; }
grep probe gpurun_out/r4/kt19.log
python3 tools/trace_split.py gpurun_out/r4/kt19 $V2
