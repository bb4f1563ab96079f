# round 4 call AF: the pipelined filter walk unrolled by two (register sets A / B swap roles, no copies
# of in-flight loads), 640 threads at 5 waves / SIMD (fu640) or 512 at 4 (fu512), against the
# against the committed build (ks7): chain / c3 / ordered / partitioned tests, then C3 walks and steps
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4af_all.log && \
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py tests/test_known_answers_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3 or partitioned or ordered" > gpurun_out/r4af_tests.log 2>&1 && \
for v in ks7 fu640 fu512 ks7 fu640 fu512; do timeout -k 10 200 python -u tools/exp_split_c3.py --lib tools/abx/libccj_$v.so c3 uni100 > gpurun_out/r4af_c3_$v.log 2>&1 && grep split gpurun_out/r4af_c3_$v.log | sed "s/^/$v /" >> gpurun_out/r4af_all.log || exit 1; done && \
for w in c3 c3o; do for v in ks7 fu640 fu512 ks7 fu640 fu512; do P=partitioned; [ $w = c3o ] && P=ordered; timeout -k 10 200 python -u bench.py --workload c3 --path $P --lib tools/abx/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4af_${w}_$v.log 2>&1 && python3 -c "
import json; d=json.loads(open('gpurun_out/r4af_${w}_$v.log').read().strip().splitlines()[-1])
print('$w $v', round(d['ms_per_step'],3), {k: round(v,3) for k, v in d.get('phases', {}).items() if isinstance(v, float)})" >> gpurun_out/r4af_all.log || exit 1; done; done
