# round 4 call AN: the split's KS (previous tile's entries stored between this tile's rankings) at
# 5 / 7 (committed) / 9 on C3's split and walk (exp_split_c3) and C2, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && rm -f gpurun_out/r4an_all.log && \
for v in ks7 ks5 ks9 ks7 ks5 ks9; do timeout -k 10 200 python -u tools/exp_split_c3.py --lib tools/abx/libccj_$v.so c3 > gpurun_out/r4an_c3_$v.log 2>&1 && grep split gpurun_out/r4an_c3_$v.log | sed "s/^/$v /" >> gpurun_out/r4an_all.log || exit 1; done && \
for v in ks7 ks5 ks9 ks7 ks5 ks9; do timeout -k 10 150 python -u bench.py --lib tools/abx/libccj_$v.so --no-cpu --no-other --no-verify --steps 10 --warmup 3 > gpurun_out/r4an_c2_$v.log 2>&1 && python3 -c "
import json,sys; d=json.loads(open('gpurun_out/r4an_c2_$v.log').read().strip().splitlines()[-1]); p=d['phases']
print('$v c2', round(d['ms_per_step'],3), round(p['hash_find_bucket_ms'],3), round(p['match_tuples_and_advance_pointers_ms'],3))" >> gpurun_out/r4an_all.log || exit 1; done
