#!/usr/bin/env python3
"""tools/overlap_part.py — experiment: the C2 probe column cut into K pieces, each a
ccj_probe_partitioned call with its own buffers, issued round-robin on S streams, so piece i's walk
(L2-request bound) can run beside piece i+1's split (HBM-store bound).  S = 1 is the same pieces in
sequence (the control).  L1/L2 of the union are checked against the exact membership answer.
Run on the GPU box:  python3 tools/overlap_part.py K/S [K/S ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import ccj  # noqa: E402


def main():
    specs = sys.argv[1:] or ["1/1", "2/1", "2/2", "4/2"]
    n_build, n_probe, chunk, seed = 1 << 26, 1 << 30, 2048, 42
    torch.cuda.set_device(0)
    ccj.device_init(0)
    s0 = torch.cuda.Stream()
    with torch.cuda.stream(s0):
        table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE, stream=s0)
        keys = ccj.gen_uniform_keys(n_probe, seed, n_build, stream=s0)
    s0.synchronize()
    from oracle import oracle as O
    want = O.count_uniform(seed, 0, n_probe, n_build, n_build, 1, threads=16)
    for spec in specs:
        k, ns = (int(x) for x in spec.split("/"))
        n = n_probe // k
        streams = [torch.cuda.Stream() for _ in range(ns)]
        pieces = []
        for i in range(k):
            st = streams[i % ns]
            with torch.cuda.stream(st):
                part = table.alloc_partitioned(n, chunk)
                out = table.alloc_outputs(part["positions"], chunk, rounds=False)
                out["status"].zero_()
            pieces.append((keys[i * n:(i + 1) * n], part, out, st))
        torch.cuda.synchronize()

        def step():
            for kk, part, out, st in pieces:
                table.probe_partitioned(kk, chunk, out=out, part=part, stream=st, retry=False)

        step()
        torch.cuda.synchronize()
        times = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s0)
            for st in streams:
                st.wait_stream(s0)
            step()
            for st in streams:
                s0.wait_stream(st)
            b.record(s0)
            torch.cuda.synchronize()
            times.append(a.elapsed_time(b))
        m_tot, l2_tot, status = 0, 0, 0
        for i, (kk, part, out, st) in enumerate(pieces):
            status |= int(out["status"].item())
            out["n_chunks"] = (part["positions"] + chunk - 1) // chunk
            rm = part["row_map"].to(torch.int64) + i * n
            m, l2 = ccj.result_checksum(out, chunk, row_map=rm, stream=st)
            torch.cuda.synchronize()
            m_tot += m
            l2_tot = (l2_tot + l2) & ((1 << 64) - 1)
            del rm
        times.sort()
        print(json.dumps({"pieces": k, "streams": ns, "ms_min": round(times[0], 3), "ms_med": round(times[2], 3),
                          "G_tuples_per_s": round(n_probe / times[2] / 1e6, 1), "status": status,
                          "l1_ok": m_tot == want[0], "l2_ok": l2_tot == want[1]}), flush=True)
        del pieces
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
