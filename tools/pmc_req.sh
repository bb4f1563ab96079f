#!/bin/bash
# Request-size / stall PMC passes for the probe (bench.py, 2 steps) and the random-read
# microbenchmark (tools/randread), one rocprofv3 --pmc pass per group.  Run on the GPU box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmc_req
mkdir -p $OUT
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"; do
  name=$(echo "$grp" | tr ' ' '+')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "probe_chunks|rand_read" -T -f csv -d $OUT/probe_$name -o pmc \
      -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-verify > $OUT/probe_$name.log 2>&1 || { echo "probe pmc $grp failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "rand_read" -T -f csv -d $OUT/rr_$name -o pmc \
      -- tools/randread > $OUT/rr_$name.log 2>&1 || { echo "randread pmc $grp failed"; exit 1; }
done
echo done
