# round 4 call Z: the split with KS = 7 as the product default: partitioned / ordered / chain /
# dist tests; KS 6-9 on C2 interleaved twice; the ordered C2 / C3 lines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4z_all.log && \
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py tests/test_dist_gpu.py tests/test_c5_gpu.py tests/test_pipeline_device_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4z_tests.log 2>&1 && \
for v in ks6 ks7 ks8 ks9 ks6 ks7 ks8 ks9; do timeout -k 10 150 python -u bench.py --lib tools/ab/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4z_$v.log 2>&1 && python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4z_$v.log').read().strip().splitlines()[-1]); p=d['phases']
print('$v', round(d['ms_per_step'],3), round(p['hash_find_bucket_ms'],3), round(p['match_tuples_and_advance_pointers_ms'],3))" >> gpurun_out/r4z_all.log || exit 1; done && \
timeout -k 10 300 python -u bench.py --path ordered --no-cpu --no-other --steps 5 --warmup 2 > gpurun_out/r4z_c2ord.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --path ordered --no-cpu --steps 5 --warmup 2 > gpurun_out/r4z_c3ord.log 2>&1 && \
timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 3 > gpurun_out/r4z_c3.log 2>&1
