# round 4 call AH: the compaction's P-stream chunk by shift (power-of-two chunks) instead of a 64-bit
# division per match (cdiv) against the committed build (ks7): compaction / c3 tests, then C3 steps
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4ah_all.log && \
timeout -k 10 600 python -u -m pytest tests/test_compact_gpu.py tests/test_c3_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4ah_tests.log 2>&1 && \
for v in ks7 cdiv ks7 cdiv ks7 cdiv; do timeout -k 10 200 python -u bench.py --workload c3 --lib tools/abx/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4ah_c3_$v.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/r4ah_c3_$v.log').read().strip().splitlines()[-1])
print('c3 $v', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d.get('phases', {}).items() if isinstance(v, float)})" >> gpurun_out/r4ah_all.log || exit 1; done
