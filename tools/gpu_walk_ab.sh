# same-box A/B of the walk's window width: CCJ_WALK_LANES 2 (32-byte windows) vs 4 (64-byte), tuning build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/walk_ab.log
for ln in 4 2 4 2; do
  CCJ_WALK_LANES=$ln timeout -k 10 200 python -u bench.py --lib tuning --no-other --no-cpu --steps 10 > gpurun_out/walk_ab_$ln.log 2>&1 || exit 1
  tail -1 gpurun_out/walk_ab_$ln.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('lanes $ln',round(d['ms_per_step'],3),d['parity']['l1_ok'],d['parity']['l2_ok'])" >> gpurun_out/walk_ab.log
done
