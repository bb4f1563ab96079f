set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r17; mkdir -p $O
for G in 8 2; do
CCJ_SHARD_GROUP=$G timeout -k 10 600 python3 bench.py --sharded --steps 3 --warmup 1 --no-cpu --no-verify > $O/sharded$G.json 2> $O/sharded$G.err || { echo "sharded failed"; tail $O/sharded$G.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/sharded$G.json'));print($G, d['ms_per_step'], d['roofline']['kernel_ms'])"
done
