# round 4 call U: the split with the previous tile's first KS entries stored between this tile's
# ranking (-DCCJ_SPLIT_KS, tools/ab/libccj_ks*.so) against KS = 0, C2 bench lines interleaved twice;
# then the filter walk with non-temporal match stores (nt) against the build without
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4u_all.log && \
for v in ks0 ks4 ks7 ks10 ks0 ks4 ks7 ks10; do timeout -k 10 150 python -u bench.py --lib tools/ab/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4u_$v.log 2>&1 && python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4u_$v.log').read().strip().splitlines()[-1]); p=d['phases']
print('$v', round(d['ms_per_step'],3), round(p['hash_find_bucket_ms'],3), round(p['match_tuples_and_advance_pointers_ms'],3))" >> gpurun_out/r4u_all.log || exit 1; done && \
timeout -k 10 400 python -u -m pytest tests/test_probe_gpu.py -x -q --timeout 300 --timeout-method thread -k "partitioned" > gpurun_out/r4u_tests.log 2>&1
