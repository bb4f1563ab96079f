# round 4 call AC: the split with per-partition full flags (one async overflow atomic per partition once
# the partition has overflowed, synchronous only the first time): partitioned / ordered / chain / c3 tests, then A/B against the
# KS = 7 build without flags on C3 (split + walk) and C2, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4ac_all.log && \
timeout -k 10 600 python -u -m pytest tests/test_probe_gpu.py tests/test_build_gpu.py tests/test_c3_gpu.py tests/test_known_answers_gpu.py -x -q --timeout 300 --timeout-method thread -k "chain or c3 or partitioned or ordered" > gpurun_out/r4ac_tests.log 2>&1 && \
for v in ks7 full ks7 full; do timeout -k 10 200 python -u tools/exp_split_c3.py --lib tools/abx/libccj_$v.so c3 > gpurun_out/r4ac_c3_$v.log 2>&1 && grep split gpurun_out/r4ac_c3_$v.log | sed "s/^/$v /" >> gpurun_out/r4ac_all.log || exit 1; done && \
for v in ks7 full ks7 full; do timeout -k 10 150 python -u bench.py --lib tools/abx/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4ac_c2_$v.log 2>&1 && python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4ac_c2_$v.log').read().strip().splitlines()[-1]); p=d['phases']
print('$v c2', round(d['ms_per_step'],3), round(p['hash_find_bucket_ms'],3), round(p['match_tuples_and_advance_pointers_ms'],3))" >> gpurun_out/r4ac_all.log || exit 1; done
