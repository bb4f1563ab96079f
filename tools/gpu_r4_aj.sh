# round 4 call AJ: C5's payload gather with cache-policy bits on its 64-byte row loads (tuning build,
# CCJ_GATHER_AUX 0 plain / 1 nt / 2 sc0 sc1 / 3 sc1 / 4 sc0): C5 steps and their phases
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4aj_all.log && \
for x in 0 1 2 3 4 0; do CCJ_GATHER_AUX=$x timeout -k 10 300 python -u bench.py --workload c5 --lib tuning --no-cpu --no-other --steps 5 --warmup 2 > gpurun_out/r4aj_c5_$x.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/r4aj_c5_$x.log').read().strip().splitlines()[-1])
print('c5 aux=$x', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d.get('phases', {}).items() if isinstance(v, float)}, d.get('parity', {}).get('columns_ok', d.get('parity')))" >> gpurun_out/r4aj_all.log || exit 1; done
