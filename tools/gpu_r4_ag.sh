# round 4 call AG: the ordered probe's walk as probe_walk2<MM> (fixed first windows, round words)
# against probe_walk1<MM>: ordered tests on the product build, then C2 ordered steps on the tuning
# build with CCJ_OWALK = 1 (walk1) / 2 (walk2, two batches) / 3 (walk2, one batch), interleaved, and
# one verified product run (equals_chunk_path_l3)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4ag_all.log && \
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_known_answers_gpu.py tests/test_pipeline_gpu.py tests/test_pipeline_device_gpu.py -x -q --timeout 300 --timeout-method thread -k "ordered or known or pipeline" > gpurun_out/r4ag_tests.log 2>&1 && \
for x in 1 2 3 1 2 3; do CCJ_OWALK=$x timeout -k 10 200 python -u bench.py --path ordered --lib tuning --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4ag_c2o_$x.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/r4ag_c2o_$x.log').read().strip().splitlines()[-1])
print('c2o owalk=$x', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d.get('phases', {}).items() if isinstance(v, float)})" >> gpurun_out/r4ag_all.log || exit 1; done && \
timeout -k 10 400 python -u bench.py --path ordered --no-cpu --no-other --steps 10 --warmup 3 > gpurun_out/r4ag_c2o_verified.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/r4ag_c2o_verified.log').read().strip().splitlines()[-1])
print('c2o product verified', round(d['ms_per_step'],3), d.get('parity'))" >> gpurun_out/r4ag_all.log
