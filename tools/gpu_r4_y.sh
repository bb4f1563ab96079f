# round 4 call Y: the split as committed (pre: stores after the reservations) against KS = 7 (the
# previous tile's first 7 entries stored between this tile's rankings), C2 lines interleaved 3x
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4y_all.log && \
for v in pre ks7 pre ks7 pre ks7; do timeout -k 10 150 python -u bench.py --lib tools/ab/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4y_$v.log 2>&1 && python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4y_$v.log').read().strip().splitlines()[-1]); p=d['phases']
print('$v', round(d['ms_per_step'],3), round(p['hash_find_bucket_ms'],3), round(p['match_tuples_and_advance_pointers_ms'],3))" >> gpurun_out/r4y_all.log || exit 1; done
