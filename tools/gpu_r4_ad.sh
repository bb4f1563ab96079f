# round 4 call AD: the unsplit in the split's XCD tile order (CCJ_UNSPLIT_XCD): ordered tests, then
# C2 / C3 ordered with the order off / on, interleaved on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4ad_all.log && \
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_c3_gpu.py tests/test_known_answers_gpu.py -x -q --timeout 300 --timeout-method thread -k "ordered or unsplit" > gpurun_out/r4ad_tests.log 2>&1 && \
for w in c2 c3; do for x in 0 1 0 1; do CCJ_UNSPLIT_XCD=$x timeout -k 10 200 python -u bench.py --workload $w --path ordered --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4ad_${w}_$x.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/r4ad_${w}_$x.log').read().strip().splitlines()[-1])
print('$w xcd=$x', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d.get('phases', {}).items() if isinstance(v, float)})" >> gpurun_out/r4ad_all.log || exit 1; done; done
