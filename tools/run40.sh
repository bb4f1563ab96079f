# GPU box: round check after the 11-key split tile — full GPU suite, smoke, default bench line, profile of that command.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r40; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed $?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail $O/bench_c2.err; exit 1; }
cut -c1-600 $O/bench_c2.json
bash tools/profile.sh r1h > $O/profile.log 2>&1 || { echo "profile failed"; tail $O/profile.log; exit 1; }
tail -1 $O/profile.log
timeout -k 10 600 python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail $O/bench_c5.err; exit 1; }
cut -c1-700 $O/bench_c5.json
timeout -k 10 600 python3 bench.py --workload c3 --steps 5 --warmup 2 --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 failed"; tail $O/bench_c3.err; exit 1; }
cut -c1-500 $O/bench_c3.json
