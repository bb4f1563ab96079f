# round 4 call X: the filter walk with per-workgroup chunk slots (LDS match counts, no device atomic
# per unit): chain / c3 / partitioned / ordered tests; C3 walk A/B against the build with the device
# atomic (tools/ab/libccj_ks0.so), interleaved twice; then the split-store interleaving A/B (KS) on C2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4x_all.log gpurun_out/r4u_all.log && \
timeout -k 10 500 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py tests/test_known_answers_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3 or partitioned or ordered" > gpurun_out/r4x_tests.log 2>&1 && \
for v in ks0 slots ks0 slots; do timeout -k 10 200 python -u tools/exp_split_c3.py --lib tools/ab/libccj_$v.so c3 > gpurun_out/r4x_$v.log 2>&1 && grep split gpurun_out/r4x_$v.log | sed "s/^/$v /" >> gpurun_out/r4x_all.log || exit 1; done && \
for v in ks0 ks4 ks7 ks10 ks0 ks4 ks7 ks10; do timeout -k 10 150 python -u bench.py --lib tools/ab/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4u_$v.log 2>&1 && python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4u_$v.log').read().strip().splitlines()[-1]); p=d['phases']
print('$v', round(d['ms_per_step'],3), round(p['hash_find_bucket_ms'],3), round(p['match_tuples_and_advance_pointers_ms'],3))" >> gpurun_out/r4u_all.log || exit 1; done
