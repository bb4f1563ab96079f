#!/bin/bash
# kernel-trace stats of one bench command per library build: tools/gpu_lib_kt.sh TAG "BENCH ARGS" LIB1 LIB2 ...
# (ON THE GPU BOX) -> gpurun_out/kt_TAG_<i>/kt_kernel_stats.csv
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; ARGS=$2; shift 2
i=0
for lib in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/kt_${TAG}_$i -o kt -- python3 bench.py --lib $lib $ARGS --no-cpu --no-verify --no-other --steps 5 --warmup 1 > gpurun_out/kt_${TAG}_$i.log 2>&1 || { echo "kt $lib failed"; tail -5 gpurun_out/kt_${TAG}_$i.log; exit 1; }
  echo "== $lib"; python3 - "$TAG" "$i" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/kt_{sys.argv[1]}_{sys.argv[2]}/kt_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e6:8.3f} ms')
PY
  i=$((i+1))
done
