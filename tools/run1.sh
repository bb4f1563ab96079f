set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 tools/l2coop > gpurun_out/l2coop.log 2>&1 || { echo "l2coop failed $?"; exit 1; }
timeout -k 10 400 python3 -u tools/sweep_part.py pair4 w1_4u_2 w1_2u_4 w1_2u_3 w1_4u_3 w1_4a_2 w1_8a_2 w2_4a_4 w2_8a_2 w2_8a_3 > gpurun_out/sweep1.log 2>&1 || { echo "sweep failed $?"; tail -20 gpurun_out/sweep1.log; exit 1; }
cat gpurun_out/sweep1.log
