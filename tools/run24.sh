set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r24; mkdir -p $O
for W in 18 19 20; do
CCJ_WINDOW_BITS=$W timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt$W -o kt -- python3 tools/sweep_part.py w2_4l_3 > $O/c2_$W.log 2>&1 || { echo "c2 failed"; tail $O/c2_$W.log; exit 1; }
python3 tools/trace_split.py $O/kt$W w$W
done
for W in 18 19; do
CCJ_WINDOW_BITS=$W timeout -k 10 600 python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu --no-verify > $O/c3_$W.json 2> $O/c3_$W.err || { echo "c3 failed"; tail $O/c3_$W.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/c3_$W.json'));print('c3 w$W', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
