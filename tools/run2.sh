# GPU box: split variants timed + kernel trace + L2/HBM request counters of the partitioned path.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r2
V="pair4/1 pair4/3 w1_2u_3/3 w2_4a_4/3 w1_4u_2/3"
timeout -k 10 300 python3 -u tools/sweep_part.py $V > gpurun_out/r2/sweep.log 2>&1 || { echo "sweep failed $?"; tail -20 gpurun_out/r2/sweep.log; exit 1; }
cat gpurun_out/r2/sweep.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r2/kt -o kt -- python3 tools/sweep_part.py $V > gpurun_out/r2/kt.log 2>&1 || { echo "kt failed $?"; exit 1; }
for grp in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"; do
  name=$(echo "$grp" | tr ' ' '+')
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "slot_split|probe_win|probe_pair" -T -f csv -d gpurun_out/r2/pmc_$name -o pmc -- python3 tools/sweep_part.py pair4/1 w1_2u_3/3 > gpurun_out/r2/pmc_$name.log 2>&1 || { echo "pmc $grp failed $?"; tail -5 gpurun_out/r2/pmc_$name.log; exit 1; }
done
echo done
