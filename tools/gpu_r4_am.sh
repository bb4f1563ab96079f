# round 4 call AM: emit_ordered re-reading the staged payload from the chunk's keys (reread: 12 KB of LDS per
# workgroup instead of 28) against the committed build (base): ordered tests on reread, then C2 / C3
# ordered steps, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4am_all.log && \
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_known_answers_gpu.py tests/test_pipeline_device_gpu.py -x -q --timeout 300 --timeout-method thread -k "ordered or known or pipeline" > gpurun_out/r4am_tests.log 2>&1 && \
for w in c2 c3; do for v in base reread base reread base reread; do timeout -k 10 200 python -u bench.py --workload $w --path ordered --lib tools/abx/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4am_${w}_$v.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/r4am_${w}_$v.log').read().strip().splitlines()[-1])
print('${w}o $v', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d.get('phases', {}).items() if isinstance(v, float)})" >> gpurun_out/r4am_all.log || exit 1; done; done
