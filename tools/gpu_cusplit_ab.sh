#!/bin/bash
# One-rank sharded rehearsal under several CU splits (ON THE GPU BOX): tools/gpu_cusplit_ab.sh "24,8" "0,0" ...
cd "$GRAFT_REPO_ROOT" || exit 1
for cs in "$@"; do
  timeout -k 10 300 python3 bench.py $BENCH_EXTRA --gpus 1 --sharded --steps 8 --warmup 2 --no-cpu --no-verify --cu-split "$cs" \
      > gpurun_out/cusplit_${cs/,/_}.log 2>&1 || { echo "cu-split $cs failed"; tail -5 gpurun_out/cusplit_${cs/,/_}.log; exit 1; }
  python3 - "$cs" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/cusplit_{sys.argv[1].replace(',', '_')}.log") if x.startswith('{"metric"')][-1]
d = json.loads(l)
print(f"cu-split {sys.argv[1]:6s} step {d['ms_per_step']:6.2f} ms  partition {d['partition_ms']:6.2f}  exchange {d['exchange_ms']:6.2f}  local probe {d['local_probe_ms']:6.2f}")
PY
done
