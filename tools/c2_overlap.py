"""Feasibility of overlapping the split of one batch with the walk of another (ON THE GPU BOX):
python3 tools/c2_overlap.py [--lib tuning]
The C2 workload (2^26-key LP table, 2^30 probes) cut into B batches of 2^30 / B keys, each one
ccj_probe_partitioned call (split + walk, CCJ_PART_ROWS) with its own workspace and outputs:
  sequential  — every batch on one stream;
  two streams — batches alternate between two streams (batch b's walk can run beside batch b+1's
                split), with and without CCJ_PART_SHARE on the splits.
Matches summed over the batches must be 2^30 either way."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd")]
import torch  # noqa: E402

import ccj  # noqa: E402

if "--lib" in sys.argv and sys.argv[sys.argv.index("--lib") + 1] == "tuning":
    ccj.LIB_PATH = os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd", "libccj_tuning.so")


def main():
    n_build, n_probe, chunk = 1 << 26, 1 << 30, 2048
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s0):
        table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE, stream=s0)
        keys = ccj.gen_uniform_keys(n_probe, 42, n_build, stream=s0)
    torch.cuda.synchronize()
    for B in (1, 2, 4, 8):
        bn = n_probe // B
        parts = [table.alloc_partitioned(bn, chunk) for _ in range(B)]
        outs = [table.alloc_outputs(p["positions"], chunk, rounds=False) for p in parts]
        torch.cuda.synchronize()

        def run(two, share):
            for b in range(B):
                st = s1 if two and b % 2 else s0
                table.probe_partitioned(keys[b * bn:(b + 1) * bn], chunk, out=outs[b], part=parts[b], stream=st,
                                        retry=False, rows=True, share=share)

        for name, two, share in (("sequential", False, False), ("two streams", True, False),
                                 ("two streams + share", True, True)):
            run(two, share)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            reps = 5
            for _ in range(reps):
                run(two, share)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / reps
            m = sum(int(o["count"][:o["n_chunks"]].sum().item()) for o in outs)
            st = max(int(o["status"].item()) for o in outs)
            print(f"B={B:2d} {name:22s} {ms:7.2f} ms per 2^30 probes  matches {m} status {st}", flush=True)
        del parts, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
