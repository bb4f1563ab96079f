# PMC passes of the C2 bench for the rank walk (one counter group per run)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pmc_rank
for grp in "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
  name=$(echo "$grp" | tr ' ' '+')
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "probe_rank|probe_walk|slot_split_pipe" -T -f csv -d gpurun_out/pmc_rank/$name -o pmc \
      -- python3 bench.py --no-other --no-cpu --no-verify --steps 2 --warmup 1 > gpurun_out/pmc_rank/$name.log 2>&1 || { echo "pmc $grp failed rc=$?"; tail -3 gpurun_out/pmc_rank/$name.log; exit 1; }
done
