# round-5 calls L / M: owner split alone (tools/owner_split_bench.py, tuning build) — forms, grids, ablations
# (0x10 no stores, 0x20 no key reads, 0x2000 no hash, 0x100000 no reservation atomics, 0x200000 no image scatter)
set -o pipefail
o=gpurun_out/${OWNER_TAG:-r5l}_owner.log  # (r5m: the first try of 0x200000 left stale image entries naming unwritten
# partition records — an out-of-bounds store; the image now starts as partition 0's entries)
: > $o
run() { echo "== $*" >> $o; env "$@" timeout -k 10 120 python3 -u tools/owner_split_bench.py --lib tuning --unmasked >> $o 2>&1; }
if [ "${OWNER_TAG:-r5l}" = r5l ]; then
run CCJ_X=0 && run CCJ_OWNER_ABLATE=16 && run CCJ_OWNER_ABLATE=32 && run CCJ_OWNER_ABLATE=8192 && run CCJ_OWNER_ABLATE=48 && \
run CCJ_OWNER_SMALL_PER_CU=0 && run CCJ_OWNER_SMALL_PER_CU=2 && run CCJ_OWNER_SMALL_PER_CU=3 && \
run CCJ_OWNER_FORM=1 && run CCJ_OWNER_FORM=2 && run CCJ_OWNER_FORM=2 CCJ_OWNER_SMALL_PER_CU=1 && run CCJ_X=0
else
run CCJ_X=0 && run CCJ_OWNER_ABLATE=1048576 && run CCJ_OWNER_SMALL=0 && run CCJ_OWNER_SMALL=0 CCJ_OWNER_WGS=256 && \
run CCJ_OWNER_ABLATE=48 && run CCJ_OWNER_ABLATE=2097152 && run CCJ_OWNER_ABLATE=3145728 && \
run CCJ_OWNER_ABLATE=3145776 && run CCJ_X=0
fi
