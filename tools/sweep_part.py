#!/usr/bin/env python3
"""tools/sweep_part.py — times ccj_probe_partitioned kernel variants on the C2 workload (2^26-key
LP table of the reference generator, 2^30 SplitMix64 probe keys, chunk 2048) after ONE setup.
CCJ_PROBE_VARIANT / CCJ_SPLIT_VARIANT (tuning overrides that libccj reads at every launch) pick
the kernels; every variant's L1/L2 answer is checked against the exact membership count.
Run on the GPU box:  python3 tools/sweep_part.py [probe_variant[/split_variant[/ablate_bits]] ...]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ccj  # noqa: E402


def main():
    specs = sys.argv[1:] or ["pair4", "w1_4u_2"]
    n_build, n_probe, chunk, seed = 1 << 26, 1 << 30, 2048, 42
    torch.cuda.set_device(0)
    ccj.device_init(0)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE, stream=stream)
        keys = ccj.gen_uniform_keys(n_probe, seed, n_build, stream=stream)
        part = table.alloc_partitioned(n_probe, chunk)
        out = table.alloc_outputs(part["positions"], chunk, rounds=False)
    stream.synchronize()
    from oracle import oracle as O
    want = O.count_uniform(seed, 0, n_probe, n_build, n_build, 1, threads=16)
    print(json.dumps({"setup": "C2", "positions": part["positions"], "expected_matches": want[0]}), flush=True)
    for spec in specs:
        pv, sv, ab = (spec.split("/") + ["", ""])[:3]
        for name, val in (("CCJ_PROBE_VARIANT", pv), ("CCJ_SPLIT_VARIANT", sv), ("CCJ_ABLATE", ab)):
            if val:
                os.environ[name] = val
            else:
                os.environ.pop(name, None)
        torch.cuda.synchronize()
        out["status"].zero_()
        torch.cuda.synchronize()

        def step():
            table.probe_partitioned(keys, chunk, out=out, part=part, stream=stream, retry=False)

        for _ in range(2):
            step()
        stream.synchronize()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in evs:
            a.record(stream)
            step()
            b.record(stream)
        stream.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in evs)
        status = int(out["status"].item())
        out["n_chunks"] = (part["positions"] + chunk - 1) // chunk
        rm = part["row_map"].to(torch.int64)
        m, l2 = ccj.result_checksum(out, chunk, row_map=rm, stream=stream)
        del rm
        print(json.dumps({"probe": pv, "split": sv or "default", "ablate": ab or "0", "ms_min": round(ms[0], 3), "ms_med": round(ms[2], 3),
                          "G_tuples_per_s": round(n_probe / ms[2] / 1e6, 1), "status": status,
                          "l1_ok": m == want[0], "l2_ok": l2 == want[1]}), flush=True)


if __name__ == "__main__":
    main()
