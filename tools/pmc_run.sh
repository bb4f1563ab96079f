#!/bin/bash
# tools/pmc_run.sh TAG REGEX -- cmd...   (on the GPU box) one rocprofv3 --pmc pass per counter group
set -o pipefail
TAG=$1; RE=$2; shift 2; [ "$1" == "--" ] && shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
for grp in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE"; do
  name=$(echo "$grp" | tr ' ' '+')
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "$RE" -T -f csv -d "gpurun_out/pmc_$TAG/$name" -o pmc \
      -- "$@" > "gpurun_out/pmc_$TAG/$name.log" 2>&1 || { echo "pmc $grp failed"; }
done
