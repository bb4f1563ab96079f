# GPU box: full GPU test suite, smoke, C2 + C5 bench lines, split grid experiment, C2 profile.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
timeout -k 10 600 python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
CCJ_SPLIT_BLOCKS=128 timeout -k 10 300 rocprofv3 --kernel-trace -T -f csv -d $O/kt128 -o kt -- python3 tools/sweep_part.py w2_4a_4 > $O/kt128.log 2>&1 || { echo "kt128 failed"; exit 1; }
python3 tools/trace_split.py $O/kt128 w2_4a_4
bash tools/profile.sh r1b > $O/profile.log 2>&1 || { echo "profile failed"; tail $O/profile.log; exit 1; }
tail -3 $O/profile.log
