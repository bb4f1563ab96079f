"""Measurement tool (not product): the partitioned chaining probe's split and walk phases on the C3
table (2^26 build keys) for several probe streams, to separate the split's cost of key skew from
its partition count.  Usage: python tools/exp_split_c3.py [--lib tuning] [streams...]
streams: c3 (Zipf hits, the bench's), c3h0 (the C3 generator's misses only: no skew), uni100 (uniform,
all hits)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd"))
import ccj  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default="product")
    ap.add_argument("--n-build", type=int, default=1 << 26)
    ap.add_argument("--n-probe", type=int, default=1 << 30)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("streams", nargs="*", default=["c3", "c3h0", "uni100"])
    a = ap.parse_args()
    if a.lib == "tuning":
        ccj.LIB_PATH = os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd", "libccj_tuning.so")
    elif a.lib != "product":
        ccj.LIB_PATH = os.path.abspath(a.lib)
    ccj.device_init(0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        table = ccj.Table.reference(ccj.CHAIN, a.n_build, 1, ccj.LAYOUT_DEVICE, stream=s)
    for name in a.streams:
        with torch.cuda.stream(s):
            if name == "c3":
                keys = ccj.gen_c3_keys(a.n_probe, 42, a.n_build, 1, stream=s)
            elif name == "c3h0":
                keys = ccj.gen_c3_keys(a.n_probe, 42, a.n_build, 1, hit_ppm=0, stream=s)
            else:
                keys = ccj.gen_uniform_keys(a.n_probe, 23, a.n_build, stream=s)
            part = table.alloc_partitioned(a.n_probe, 2048)
            out = table.alloc_outputs(part["positions"], 2048, rounds=False)
        s.synchronize()
        pev = [ccj.PhaseEvents() for _ in range(a.steps + 1)]
        for pe in pev:
            pe.arm()
            table.probe_partitioned(keys, 2048, out=out, part=part, stream=s, retry=False)
            ccj.PhaseEvents.disarm()
        s.synchronize()
        t = [pe.ms() for pe in pev[1:]]
        split = sum(x[0] for x in t) / len(t)
        walk = sum(x[1] for x in t) / len(t)
        st = int(out["status"].item())
        print(f"{name:7s} split {split:.3f} ms  walk {walk:.3f} ms  status {st:#x}  "
              f"matches {int(out['count'].sum().item())}", flush=True)
        del keys, part, out


if __name__ == "__main__":
    main()
