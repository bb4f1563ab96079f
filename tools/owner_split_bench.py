"""Owner split alone (ON THE GPU BOX): ms per 2^25-key batch of ccj_partition_by_owner_grouped for
1, 2, 4 and 8 owners, on an unmasked stream (the default half-CU grid) and on CU-masked streams of 64 / 128
CUs (one workgroup per CU), nothing else running.  python3 tools/owner_split_bench.py [--lib tuning|PATH]
[--unmasked].  Tuning-build knobs: CCJ_OWNER_DIRECT=0 (round 4's slot_split_pipe form),
CCJ_OWNER_RANK=0 (owner_split_direct's ballot ranking at every owner count),
CCJ_OWNER_PER_CU (persistent workgroups per CU; 0: one per tile), CCJ_OWNER_ABLATE (0x10 no stores,
0x20 no key reads, 0x2000 no hash, 0x100000 no reservation atomics, 0x200000 no image scatter;
the last two in the round-4 form)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd")]
import torch  # noqa: E402

import ccj  # noqa: E402

if "--lib" in sys.argv:  # tuning, or the path of another build (A/B)
    _lib = sys.argv[sys.argv.index("--lib") + 1]
    ccj.LIB_PATH = (os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd", "libccj_tuning.so")
                    if _lib == "tuning" else os.path.abspath(_lib))


def run(parts, stream, n=1 << 25, iters=20):
    keys = ccj.gen_uniform_keys(n, 42, 1 << 27, first_row=0)
    sub = ccj.grouped_sub_cap(n, parts, 2048)
    p = ccj.GroupedOwnerPartitioner(n, parts, sub)
    ok = torch.empty(parts * 8 * sub, dtype=torch.int64, device="cuda")
    orr = torch.empty(parts * 8 * sub, dtype=torch.int32, device="cuda")
    oc = torch.empty(parts * 8, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(3):
        p(keys, 0, ok, orr, oc, st, stream=stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record(stream)
    for _ in range(iters):
        p(keys, 0, ok, orr, oc, st, stream=stream)
    b.record(stream)
    torch.cuda.synchronize()
    if not os.environ.get("CCJ_OWNER_ABLATE"):  # (timing ablations write wrong outputs)
        assert int(oc.sum().item()) == n and int(st.item()) == 0
    return a.elapsed_time(b) / iters


def main():
    print({k: v for k, v in os.environ.items() if k.startswith("CCJ_")})
    streams = {"unmasked": torch.cuda.Stream(),
               "masked 64 CUs": ccj.cu_masked_stream(ccj.cu_mask_groups(set(range(24, 32)))),
               "masked 128 CUs": ccj.cu_masked_stream(ccj.cu_mask_groups(set(range(16, 32))))}
    if "--unmasked" in sys.argv:
        streams = {k: v for k, v in streams.items() if k.startswith("unmasked")}
    for parts in (1, 2, 4, 8):
        for name, s in streams.items():
            ms = run(parts, s)
            print(f"owners {parts}  {name:24s} {ms:7.3f} ms per 2^25 keys  ({(1 << 25) * 20 / ms / 1e6:7.1f} GB/s of 20 B/key)")


if __name__ == "__main__":
    main()
