#!/bin/bash
# tools/gpu_ab.sh TAG WORKLOAD REPS VARIANT... — same-box A/B, run ON THE GPU BOX (via gpurun).
# Replaces round 4's one-off tools/gpu_r4_*.sh scripts.  Each VARIANT is LIB or LIB:ENV=V[,ENV=V]:
# LIB = "product", "tuning" or a library path (a build of libccj with one change, e.g.
# tools/abx/libccj_<name>.so, a git-ignored directory that travels to the box), ENV the tuning build's environment overrides for that run.  The variants run interleaved REPS times; one
# summary line per run goes to gpurun_out/TAG_all.log:
#   WORKLOAD c2 | c2ord | c3 | c5: bench.py's line — ms per step and the phases (split / walk / gather)
#   WORKLOAD c3split:              tools/exp_split_c3.py's split + walk lines
# Every run under its own time limit; the first failure ends the script (no retries).
TAG=$1; WL=$2; REPS=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out && rm -f "gpurun_out/${TAG}_all.log"
for ((r = 0; r < REPS; r++)); do
  for v in "$@"; do
    lib=${v%%:*}; envs=""
    case $v in
      *:*) envs=$(echo "${v#*:}" | tr ',' ' ') ;;
    esac
    name=$(echo "$v" | tr '/:=,' '____')
    log="gpurun_out/${TAG}_${name}_${r}.log"
    case $WL in
      c3split) env $envs timeout -k 10 200 python -u tools/exp_split_c3.py --lib "$lib" c3 > "$log" 2>&1 || exit 1
               grep split "$log" | sed "s|^|$v |" >> "gpurun_out/${TAG}_all.log" ;;
      *) args="--no-cpu --no-other --no-other-workloads --no-scaling-reference --no-verify --steps 10 --warmup 3"
         case $WL in c2ord) args="$args --path ordered" ;; c3) args="$args --workload c3" ;; c5) args="$args --workload c5" ;; esac
         env $envs timeout -k 10 200 python -u bench.py --lib "$lib" $args > "$log" 2>&1 || exit 1
         python3 - "$log" "$v" >> "gpurun_out/${TAG}_all.log" <<'PY' || exit 1
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d["phases"]
print(sys.argv[2], round(d["ms_per_step"], 3), "split", round(p["hash_find_bucket_ms"], 3), "walk",
      round(p["match_tuples_and_advance_pointers_ms"], 3), "gather", round(p["gather_tuples_ms"], 3))
PY
      ;;
    esac
  done
done
cat "gpurun_out/${TAG}_all.log"
