#!/usr/bin/env python3
"""bench.py — probe throughput of the MI355X hash-join hot path (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c3|c5|pipeline] [--no-cpu]
  N > 1: `python bench.py --gpus N` starts its own N rank processes (torch.distributed.run as a child
  process, before any GPU call in this one) and forwards rank 0's JSON line; launched by an outside
  torchrun (WORLD_SIZE set) it runs as that rank directly.

Step = one pass of the hot path over one batch:
  c2 (default; BASELINE configs[1]): LP table of 2^26 reference-generator keys (2 GiB, alpha 1/4),
      2^30 uniform probe keys in [0, 2^26) resident in HBM, chunk 2048 -> one ccj_probe launch
      (hash, probe rounds, ballot packs, payload) writing row ids + payloads + per-round counts.
  c3 (BASELINE configs[2]): chaining table of 2^26 reference keys, 2^30 probe keys with ~10 %
      Zipf-skewed hits (ccj_gen_c3_keys), chunk 2048; a step = probe + compaction of every Next
      result (the selection-vector pack stress case).
  c5 (BASELINE configs[4]): C2 plus 8 int64 build-side payload columns p_c = k*(c+1)+c, gathered
      on every match (position-major payload rows: one 64-byte row read per match).
  pipeline: main.cpp's default 3-join pipeline (2e7 LHS rows, 2e6-key chaining tables, cf 1,
      B 256, main.cpp's own mt19937(2) data) on the device (ccj_pipeline_run, host/ccj_pipeline
      --engine batched) with the compactor between joins, no-compaction timed beside it.
  N > 1 (C4 shape, weak scaling): every rank owns the build keys with owner = h(k) >> (64-log2 N)
      and 2^30 probe keys of its own; a step = owner partition + RCCL all-to-all (xGMI) + local
      probe.
Prints ONE JSON line on rank 0 with roofline and cpu_baseline objects.
The default c2 line also carries `other_workloads`: C3 and C5 timed in the same run, each with its
own parity checks and roofline (--no-other-workloads skips them).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ccj  # noqa: E402

METRIC = "probe tuples/sec + achieved HBM GB/s, 1B-row int64 join at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
SEED = 42
PATH_KERNELS = {
    "partitioned": "ccj_probe_partitioned, CCJ_PART_ROWS (slot_split_pipe writing keys + rows into the outputs, probe_walk2: one lane per row, LDS-DMA table windows, a row ends at its match (distinct keys))",
    "rank": "ccj_probe_partitioned, CCJ_PART_ROWS | CCJ_PART_RANK (slot_split_pipe + probe_rank: the window's occupancy "
            "bitmap + rank in LDS, keys from the compact array; rank_finish) — opt-in, A/B",
    "ordered": "ccj_probe_ordered (slot_split_pipe with runs + probe_walk1<1,MM> + unsplit_words + emit_ordered, 16-bit round words)",
    "chunk": "ccj_probe (probe_chunks<LP,2>)",
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c2", "c3", "c5", "pipeline"])
    ap.add_argument("--batches", type=int, default=4, help="N > 1: exchange batches per step (pipelined)")
    ap.add_argument("--group", type=int, default=None,
                    help="N > 1: received batches per local probe (each local probe sweeps the whole table); "
                         "default ccj_dist.GROUP")
    ap.add_argument("--part-share", default="on", choices=["on", "off"],
                    help="N > 1 step: the local probe's split on 3/4 of the CUs (room for the exchange's RCCL "
                         "kernels and the next owner splits)")
    ap.add_argument("--cu-split", default=None,
                    help="N > 1: 'P,Q' = groups of 8 CUs (of 32) for the local probe's and the owner split's "
                         "streams (the rest stay free for RCCL); '0,0' = unmasked; default ccj_dist.CU_SPLIT")
    ap.add_argument("--ops-module", default=None,
                    help=argparse.SUPPRESS)  # tests only: a module whose make_ops() replaces the HIP ops (CPU, gloo)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"], help=argparse.SUPPRESS)
    # tests only: every rank on cuda:0 (with --backend gloo: the N > 1 HIP path rehearsed on a one-GPU
    # box, the exchanges staged through the host by gloo instead of RCCL over xGMI)
    ap.add_argument("--same-device", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--sharded", action="store_true",
                    help="run the N > 1 protocol (through the same self-launcher) even at N = 1 (rehearsal)")
    ap.add_argument("--pipe-lhs", type=int, default=20000000)
    ap.add_argument("--pipe-rhs", type=int, default=2000000)
    ap.add_argument("--pipe-joins", type=int, default=3)
    ap.add_argument("--pipe-block", type=int, default=256)
    ap.add_argument("--pipe-table", default="chain", choices=["chain", "lp"])
    ap.add_argument("--n-build", type=int, default=1 << 26, help="N = 1: build keys (C2)")
    ap.add_argument("--n-build-per-gpu", type=int, default=1 << 27,
                    help="N > 1: build keys per GPU (C4: 2^30 total at 8 GPUs)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = --n-probe keys per GPU (C4), strong = --n-probe keys in total")
    ap.add_argument("--n-probe", type=int, default=1 << 30, help="probe keys per GPU")
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--layout", default="device", choices=["device", "reference"])
    ap.add_argument("--path", default="partitioned", choices=["partitioned", "chunk", "ordered"],
                    help="partitioned: slot-range partition + L2-resident probe (L1/L2 parity); "
                         "chunk: reference-order chunk probe (L3 parity)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-sample", type=int, default=1 << 28, help="probe keys in the multi-thread CPU sample")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-other", action="store_true", help="C2: do not time the other paths beside the headline")
    ap.add_argument("--no-other-workloads", action="store_true",
                    help="C2: do not run C3 and C5 after the headline (other_workloads)")
    ap.add_argument("--no-scaling-reference", action="store_true",
                    help="C2: do not run the multi-GPU protocol at N = 1 on the C4 per-GPU shape (scaling_reference)")
    ap.add_argument("--no-n1-same-shape", action="store_true",
                    help="N > 1: do not time the same per-GPU shape at N = 1 (n1_same_shape_ms)")
    ap.add_argument("--no-rows", action="store_true",
                    help="partitioned path without CCJ_PART_ROWS (the walk writes every output; A/B)")
    ap.add_argument("--lib", default="product",
                    help="product | tuning (libccj_tuning.so: make tuning; A/B sweeps with its env overrides) | "
                         "a path to another build of the library (same-box A/B of two source versions)")
    a = ap.parse_args()
    if a.lib == "tuning":
        ccj.LIB_PATH = os.path.join(PKG, "libccj_tuning.so")
    elif a.lib != "product":
        ccj.LIB_PATH = os.path.abspath(a.lib)
    return a


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def copy_ceiling(dev, stream, nbytes=4 << 30, iters=10):
    """Measured HBM copy ceiling: GB/s of bytes read + written by ccj_copy_device
    (16-byte non-temporal loads/stores) over a 4 GiB buffer, with torch's copy_ beside it."""
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty_like(src)
    res = {"bytes_per_copy": nbytes, "iters": iters}
    for name, fn in (("ccj_copy_device", lambda: ccj.copy_device(dst, src, stream=stream)),
                     ("torch_copy", lambda: dst.copy_(src))):
        st = stream if name == "ccj_copy_device" else torch.cuda.current_stream()
        fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(st)
        for _ in range(iters):
            fn()
        b.record(st)
        torch.cuda.synchronize()
        res[f"{name}_GBps"] = 2 * nbytes * iters / (a.elapsed_time(b) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    res["GBps"] = max(res["ccj_copy_device_GBps"], res["torch_copy_GBps"])
    return res


def physical_cores():
    """Distinct (socket, core) pairs in /proc/cpuinfo (the host's physical cores), or None."""
    try:
        cores, phys = set(), None
        for line in open("/proc/cpuinfo"):
            if line.startswith("physical id"):
                phys = line.split(":", 1)[1].strip()
            elif line.startswith("core id"):
                cores.add((phys, line.split(":", 1)[1].strip()))
        return len(cores) or None
    except OSError:
        return None


def cpu_share():
    """CPUs this process may use (the GPU box grants one GPU's share of the host: 16)."""
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count()


REF_DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")


def has_avx512():
    try:
        return "avx512f" in open("/proc/cpuinfo").read()
    except OSError:
        return False


def reference_cpu(args, n):
    """The reference's own LP Probe + Next loop (linear_probing_ht.cpp, compiled from its sources
    into oracle/_ref/ref_driver by oracle/Makefile), single thread, on the first n keys of the
    same probe stream; returns (tuples/s, seconds, matches, wall incl. build) or None."""
    import subprocess
    if not (os.path.exists(REF_DRIVER) and has_avx512()):
        return None
    t0 = time.perf_counter()
    p = subprocess.run([REF_DRIVER, "bench", "lp", "next", str(args.chunk), str(args.n_build), "1", str(n),
                        str(args.n_build), str(SEED)], capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        log(f"[cpu] reference driver failed: {p.stderr[-300:]}")
        return None
    t = p.stdout.split()
    i = t.index("BENCH")
    m, secs = int(t[i + 2]), float(t[i + 4])
    return n / secs, secs, m, time.perf_counter() - t0


def cpu_baseline(args):
    """The reference's scalar CPU path timed on this box's host cores, on a bounded sample of the
    same workload: the reference's own code (oracle/_ref, kind "reference", 1 core — it is
    single-threaded) when it is present, plus our C restatement (oracle/, "port") multi-threaded."""
    from oracle import oracle as O

    t0 = time.perf_counter()
    table = O.Table(O.LP, O.ref_build_keys(args.n_build, 1))
    build_s = time.perf_counter() - t0
    res = {}
    for threads, n in ((1, args.cpu_sample // 8), (args.cpu_threads, args.cpu_sample)):
        keys = O.uniform_keys(SEED, 0, n, args.n_build, threads=args.cpu_threads)
        table.probe_totals(keys[: 1 << 16], args.chunk, threads=threads)  # warm
        t0 = time.perf_counter()
        m, l2 = table.probe_totals(keys, args.chunk, threads=threads)
        dt = time.perf_counter() - t0
        res[threads] = (n / dt, n, dt, m)
    del table
    thr = args.cpu_threads
    v, n, dt, m = res[thr]
    v1, n1, dt1, _ = res[1]
    port = {
        "value": v, "unit": "probe tuples/s", "cores": thr, "kind": "port",
        "host": {"cpu_model": cpu_model(), "logical_cpus": os.cpu_count(), "physical_cores": physical_cores(),
                 "cpus_granted": cpu_share(),
                 "note": ("the GPU box grants one GPU's share of the host's CPUs (OMP_NUM_THREADS / MAX_JOBS = 16 "
                          "there; at most that many worker processes or threads are allowed), so the port runs "
                          "--cpu-threads (16) threads, not every physical core")},
        "sample": (f"first {n} of the same 2^30-key uniform probe stream (seed {SEED}) against the same "
                   f"{args.n_build}-key LP table built on the host, chunk {args.chunk}, {thr} threads "
                   f"(one per contiguous chunk range), {dt:.2f} s; 1 thread on {n1} keys: "
                   f"{v1 / 1e6:.1f} M tuples/s ({dt1:.2f} s); table build {build_s:.1f} s untimed"),
        "single_thread_value": v1,
    }
    n_ref = args.cpu_sample // 2
    ref = reference_cpu(args, n_ref)
    if ref is None:
        port.update(cpu_model=cpu_model(), nproc=os.cpu_count())
        return port
    rv, rs, rm, rwall = ref
    return {
        "value": rv, "unit": "probe tuples/s", "cores": 1, "kind": "reference",
        "sample": (f"the reference's LPHashTable(2^26, 1) + Probe/Next loop (its sources compiled by "
                   f"oracle/Makefile, -O3 AVX-512), one thread, on the first {n_ref} keys of the same "
                   f"probe stream (seed {SEED}), chunk {args.chunk}: {rs:.2f} s timed, {rm} matches "
                   f"(expected {n_ref}); table build + key generation untimed ({rwall - rs:.1f} s)"),
        "matches_ok": rm == n_ref,
        "port_multithread": port,
        "cpu_model": cpu_model(),
        "nproc": os.cpu_count(),
    }


def profile_traffic(workload, path, n_probe, n_build):
    """HBM bytes per step of a path's kernels from its committed counter profile
    (profiles/pmc_<workload>_<path>.json, tools/profile.sh + tools/prof_summary.py), used only when
    the profile was taken on this shape AND on the build this process loaded (its csrc_hash equals
    ccj_build_hash): a profile of an older kernel is reported as stale with traffic null."""
    res = {"traffic": None, "kernels_ms": None, "profile": None, "profile_tag": None, "profile_csrc_hash": None,
           "traffic_stale": None}
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{workload}_{path}.json")
    if not os.path.exists(pmc_path):
        return res
    try:
        pmc = json.load(open(pmc_path))
    except (OSError, ValueError):
        return res
    res.update(profile=os.path.relpath(pmc_path, ROOT), profile_tag=pmc.get("tag"),
               profile_csrc_hash=pmc.get("csrc_hash"))
    if pmc.get("n_probe") != n_probe or pmc.get("n_build") != n_build:
        return res
    stale = pmc.get("csrc_hash") != ccj.build_hash()
    res["traffic_stale"] = stale
    if not stale:
        res.update(traffic=pmc.get("hbm_bytes_per_launch"), kernels_ms=pmc.get("kernels_ms"))
    return res


PHASE_KERNELS = {  # which kernels sit between the phase boundaries of each path (ccj.h ccj_set_phase_events)
    "partitioned": ("slot_split_pipe (hash, home partition, keys + rows to their positions)",
                    "probe_walk2 (match + advance, fused; compacts the chunks with misses)",
                    "— (the split wrote the payload: it IS the probe key at its position)"),
    "ordered": ("slot_split_pipe with run records", "probe_walk1<1,MM> / chain_words (round words)",
                "unsplit_words + emit_ordered (the reference's per-Next order)"),
    "chunk": ("probe_chunks (fused: hash, match, gather, advance in one kernel)", "—", "—"),
    "rank": ("slot_split_pipe", "probe_rank + rank_finish", "—"),
}


def phase_report(pev, path, c5=False):
    """Mean per-step phase times in the reference's 4-phase schema (CycleProfiler, profiler.h:262-290:
    "Hash & Find Bucket", "Match Tuples", "Gather Tuples", "Advance Pointers") from the HIP events the
    library recorded at its kernel boundaries.  The walks fuse Match and Advance (one kernel), so they
    are reported as one phase."""
    t = [p.ms() for p in pev]
    mean = [sum(x[i] for x in t) / len(t) for i in range(3)]
    k = PHASE_KERNELS.get(path, ("?", "?", "?"))
    gather_k = (ccj.last_gather_kernel() or "?") if c5 else k[2]
    return {"schema": "reference CycleProfiler phases (profiler.h:262-290)",
            "hash_find_bucket_ms": mean[0], "match_tuples_and_advance_pointers_ms": mean[1],
            "gather_tuples_ms": mean[2],
            "kernels": {"hash_find_bucket": k[0], "match_tuples_and_advance_pointers": k[1],
                        "gather_tuples": gather_k}}


def bench_c3(args, dev, stream):
    """C3: chaining probe + NaiveCompactor under Zipf-skewed keys with ~10 % matches."""
    import subprocess
    n_build, n_probe, chunk = args.n_build, args.n_probe, args.chunk
    t0 = time.perf_counter()
    part_mode = args.path == "partitioned"
    part = pkeys = ws_o = None
    with torch.cuda.stream(stream):
        table = ccj.Table.reference(ccj.CHAIN, n_build, 1, ccj.LAYOUT_DEVICE, stream=stream)
        keys = ccj.gen_c3_keys(n_probe, SEED, n_build, 1, stream=stream)
        if part_mode:  # bucket-range split + L2-resident chain walk; one compactor input per chunk
            part = table.alloc_partitioned(n_probe, chunk)
            out = table.alloc_outputs(part["positions"], chunk, rounds=False)
            out["max_rounds"] = 1
            pkeys = part["ws"][:part["positions"] * 8].view(torch.int64)  # the partitioned key column
        else:  # chunk / ordered: the reference's Next results (round-major per chunk), compacted as such
            out = table.alloc_outputs(n_probe, chunk, rounds=True)
            if args.path == "ordered":
                ws_o = table.alloc_ordered(n_probe, chunk)
    stream.synchronize()
    log(f"[setup c3] {table.size} buckets, max chain {table.max_rounds}: {time.perf_counter() - t0:.1f} s")
    comp = None
    comp_in = {}  # partitioned: the probe outputs plus one Next result per chunk, for the compactor

    def step(ev=None, pe=None):
        nonlocal comp
        if ev:
            ev[0].record(stream)
        if pe:
            pe.arm()
        if part_mode:
            # one-pass split: the Zipf-hot keys' runs that overflow their segments go to the shared
            # overflow area; status is checked after the timed region (no host sync inside it)
            table.probe_partitioned(keys, chunk, out=out, part=part, stream=stream, retry=False)
            with torch.cuda.stream(stream):  # partition order has no Next boundaries: one result per chunk
                # (in the compactor's view only: the probe itself is asked for no rounds)
                comp_in.update(out, rounds=(out["count"] > 0).to(torch.int32), round_counts=out["count"])
        elif args.path == "ordered":  # L3 through the bucket-partitioned layout (status read after timing)
            table.probe_ordered(keys, chunk, out=out, ws=ws_o, stream=stream, retry=False)
        else:
            table.probe(keys, chunk, out=out, stream=stream)
        if ev:
            ev[1].record(stream)
        if pe:
            ccj.PhaseEvents.disarm()
        # the carried probe column is the join key: filled from the payload (equal on every match;
        # include/ccj.h ccj_compact_args.key_cols) — the gathered form is timed beside (untimed here)
        comp = ccj.compact(comp_in if part_mode else out, chunk, cols=[pkeys if part_mode else keys], rows=True,
                           stream=stream, key_cols=[0])
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    stream.synchronize()
    torch.cuda.synchronize()
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    pev = [ccj.PhaseEvents() for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i], pev[i])
    stream.synchronize()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    probe_ms = sum(a.elapsed_time(b) for a, b, _ in evs) / args.steps
    comp_ms = sum(b.elapsed_time(c) for _, b, c in evs) / args.steps
    # the general compaction (every carried column gathered through the selection vector, as
    # DataChunk::Append does), timed after the steps on the last step's probe output
    gev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(2)) for _ in range(3)]
    for a, b in gev:
        a.record(stream)
        g = ccj.compact(comp_in if part_mode else out, chunk, cols=[pkeys if part_mode else keys], rows=True,
                        stream=stream)
        b.record(stream)
    stream.synchronize()
    comp_gather_ms = min(a.elapsed_time(b) for a, b in gev)
    phases = phase_report(pev, args.path)
    phases["compaction_ms"] = comp_ms
    phases["compaction_gather_ms"] = comp_gather_ms
    phases["kernels"]["compaction"] = ("ccj_compact (NaiveCompactor closed form: scans + copy_rows_flat; the "
                                       "carried join-key column filled from the payload, key_cols)")
    phases["kernels"]["compaction_gather"] = "ccj_compact with the key column gathered by sel (DataChunk::Append's form)"
    if part_mode:
        phases["kernels"]["match_tuples_and_advance_pointers"] = (
            "probe_chain_filt (the partition's 2-bit bucket filter in LDS, 8-byte fingerprinted bucket records; "
            "probe_chain_win<3> for the overflow area's chunks)")
        phases["kernels"]["gather_tuples"] = "— (the walk writes each match's payload)"
    if part_mode or args.path == "ordered":
        if int(out["status"].item()) & ccj.FLAG_PART_OVERFLOW:
            raise SystemExit("bench c3: the split's overflow area overflowed")
    if part_mode:
        matches, l2 = ccj.result_checksum(out, chunk, row_map=part["row_map"].to(torch.int64), stream=stream)
    else:
        matches, l2 = ccj.result_checksum(out, chunk, stream=stream)
    # the compacted chunks themselves: every (row, payload) pair and the carried key column
    torch.cuda.synchronize()
    n_oc = int(comp["n"].item())
    cnt = comp["counts"][:n_oc].to(torch.int64)
    valid = (torch.arange(chunk, device=cnt.device)[None, :] < cnt[:, None]).reshape(-1)
    idx = torch.nonzero(valid).squeeze(1)
    c_rows, c_pay, c_key = comp["row"][idx], comp["payload"][idx], comp["cols"][0][idx]
    if part_mode:
        c_rows = part["row_map"].to(torch.int64)[c_rows]
    n_comp = int(idx.numel())
    key_ok = bool(torch.equal(c_key, c_pay))  # the carried key column == the matched key
    # the gathered form (DataChunk::Append through sel) gives the same key column, row for row
    g_ok = int(g["n"].item()) == n_oc and bool(torch.equal(g["cols"][0][idx], c_key))
    del g
    comp_l2 = None
    if not args.no_verify:  # checker only (the oracle's L2 term), untimed
        from oracle import oracle as O
        comp_l2 = O.l2_sum(c_rows.cpu().numpy().astype(np.uint64), c_pay.cpu().numpy())
    del c_rows, c_pay, c_key, idx, valid
    examined, _, walked, windows = table.probe_cost_walk(keys, stream=stream)
    parity = {"status_flags": int(out["status"].item()) | int(comp["status"].item()), "matches": matches,
              "l2": hex(l2), "compacted_rows": n_comp, "compacted_l2": None if comp_l2 is None else hex(comp_l2),
              "compaction_keeps_all": n_comp == matches and key_ok and comp_l2 in (None, l2),
              "gathered_key_column_equal": g_ok}
    cpu = None
    if not args.no_verify or not args.no_cpu:
        from oracle import oracle as O
        if not args.no_verify:
            want = O.count_c3(SEED, 0, n_probe, n_build, 1, threads=args.cpu_threads)
            parity.update(expected_matches=want[0], l1_ok=want[0] == matches, l2_ok=want[1] == l2)
        if not args.no_cpu and os.path.exists(REF_DRIVER) and has_avx512():
            n_ref = args.cpu_sample // 4
            p = subprocess.run([REF_DRIVER, "bench", "chain", "next", str(chunk), str(n_build), "1", str(n_ref),
                                str(n_build), str(SEED), "c3"], capture_output=True, text=True, timeout=600)
            t = p.stdout.split()
            if p.returncode == 0 and "BENCH" in t:
                rm, rs = int(t[t.index("BENCH") + 2]), float(t[t.index("BENCH") + 4])
                want_ref = O.count_c3(SEED, 0, n_ref, n_build, 1, threads=args.cpu_threads)[0]
                cpu = {"value": n_ref / rs, "unit": "probe tuples/s", "cores": 1, "kind": "reference",
                       "sample": (f"the reference's HashTable({n_build}, 1) + Probe/Next loop (chaining_ht.cpp, compiled "
                                  f"from its sources), one thread, on the first {n_ref} keys of the same C3 stream: "
                                  f"{rs:.2f} s, {rm} matches (expected {want_ref})"),
                       "matches_ok": rm == want_ref, "cpu_model": cpu_model()}
    n_bar, m_bar = examined / n_probe, matches / n_probe
    # SURVEY §8(d) for chaining: 8 (probe key) + 4 (bucket offset) + 8·N̄ (chain keys visited) +
    # 12·m̄ (u32 row id + payload per match); the step also compacts every match (NaiveCompactor,
    # compactor.cpp:5-41): per match it reads the row id (4) and payload (8) and writes the dense
    # u64 row (8), the carried key column (8) and the payload (8) = 36 B.  frac = those bytes over
    # the step's kernel time, probe + compaction.
    alg_probe = 8 + 4 + 8 * n_bar + 12 * m_bar
    alg_compact = 36 * m_bar
    alg = alg_probe + alg_compact
    step_kern_ms = probe_ms + comp_ms
    prof = profile_traffic("c3", args.path, n_probe, n_build)  # DRAM bytes of the probe kernels per step
    c3_traffic = prof["traffic"]
    achieved = alg * n_probe / (step_kern_ms * 1e-3) / 1e9
    # round 5's figure (kept as frac_csr): both CSR offsets (8 B) and no compaction, over the probe alone
    alg_csr = 8 + 8 + 8 * n_bar + 12 * m_bar
    achieved_csr = alg_csr * n_probe / (probe_ms * 1e-3) / 1e9
    # the chain keys a walk that stops at the first match examines (distinct build keys: the
    # partitioned walk)
    fm = part_mode and int(table.max_dup) <= 1
    n_walk = (walked if fm else examined) / n_probe
    alg_walked = 8 + 4 + 8 * n_walk + 12 * m_bar + alg_compact
    achieved_walked = alg_walked * n_probe / (step_kern_ms * 1e-3) / 1e9
    line = {
        "metric": METRIC, "value": n_probe / (wall / args.steps), "unit": "probe tuples/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic (reference key generator build side; C3 stream: 10 % hits, Zipf s = 1 over the 2^26 build ranks (2^16-bucket inverse CDF), seed 42)",
        "config": {"workload": "C3: 1xMI355X chaining_ht + compactor, Zipf-skewed keys, ~10% match rate, "
                               f"{n_build} build / {n_probe} probe, chunk={chunk}", "parallelism": "dp1"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "frac_basis": ("SURVEY §8(d): 8 + 4 + 8·N̄ + 12·m̄ per probe tuple, + 36·m̄ of compaction, over "
                                    "the step's kernel time (probe + compaction)"),
                     "traffic": c3_traffic,
                     "traffic_scope": "DRAM bytes per step of the probe kernels (split + walk), not the compaction",
                     "traffic_profile": prof["profile"], "traffic_profile_tag": prof["profile_tag"],
                     "traffic_profile_csrc_hash": prof["profile_csrc_hash"], "traffic_stale": prof["traffic_stale"],
                     "traffic_GBps": c3_traffic / (probe_ms * 1e-3) / 1e9 if c3_traffic else None,
                     "kernel": ("ccj_probe_partitioned (bucket-range split + probe_chain_filt) + ccj_compact" if part_mode
                                else "ccj_probe_ordered (bucket split with runs + chain_words_filt + unsplit_words + "
                                     "emit_ordered<CHAIN>) + ccj_compact" if args.path == "ordered"
                                else "probe_chunks<CHAIN,2> + ccj_compact"),
                     "kernel_ms": step_kern_ms, "probe_kernel_ms": probe_ms, "compaction_kernel_ms": comp_ms,
                     "alg_bytes_per_tuple": alg, "alg_probe_bytes_per_tuple": alg_probe,
                     "alg_compaction_bytes_per_tuple": alg_compact, "chain_keys_per_tuple": n_bar,
                     "frac_csr": achieved_csr / HBM_PEAK_GBS,
                     "frac_csr_basis": "8 + 8 + 8·N̄ + 12·m̄ (both CSR offsets) over the probe kernels alone (round 5's figure)",
                     "m_bar": m_bar, "frac_walked": achieved_walked / HBM_PEAK_GBS,
                     "alg_bytes_walked_per_tuple": alg_walked, "chain_keys_walked_per_tuple": n_walk,
                     "walk": "first match" if fm else "whole chain",
                     "chain_windows_per_tuple": windows / n_probe},
        "phases": phases,
        "compaction_ms": comp_ms, "path": args.path,
        "cpu_baseline": cpu,
        "parity": parity,
    }
    return line


def bench_pipeline(args):
    """main.cpp's pipeline on the device (host/ccj_pipeline --engine batched -> ccj_pipeline_run)
    with and without compaction, and the reference's own pipeline on the host CPU, same data."""
    import subprocess
    binp = os.path.join(PKG, "host", "ccj_pipeline")
    reps = args.warmup + args.steps
    spec = [str(x) for x in ("--join-num", args.pipe_joins, "--chunk-factor", 1, "--lhs-size", args.pipe_lhs,
                             "--rhs-size", args.pipe_rhs, "--table", args.pipe_table,
                             "--block-size", args.pipe_block, "--engine", "batched", "--repeat", reps)]
    runs = {}
    for mode in ("full", "none", "dynamic"):
        extra = ["--compact", mode]
        if mode == "dynamic":  # the UCB tuner needs its warm-up (4 pulls per arm) before it settles
            extra += ["--repeat", str(max(reps, 100))]
        p = subprocess.run([binp] + spec + extra, capture_output=True, text=True, timeout=900)
        if p.returncode != 0:
            raise RuntimeError(f"ccj_pipeline failed: {p.stderr[-500:]}")
        out = {}
        for line in (p.stdout + p.stderr).splitlines():
            t = line.split()
            if t and t[0] == "PIPE":
                out["n_out"], out["l2"] = int(t[2]), int(t[4])
            elif t and t[0] == "TIMES":
                out["times"] = [float(x) for x in t[1:]]
            elif t and t[0] == "[join":
                out.setdefault("joins", []).append({t[i]: (float(t[i + 1]) if t[i] == "ms" else int(t[i + 1]))
                                                    for i in range(2, len(t), 2)})
            elif t and t[0] == "TUNER":
                out.setdefault("tuner", []).append(" ".join(t[3:]))
        tt = out["times"][args.warmup:] if mode != "dynamic" else out["times"][-args.steps:]
        out["s_per_step"] = sum(tt) / len(tt)
        runs[mode] = out
        log(f"[pipeline] {mode}: {out['s_per_step'] * 1e3:.2f} ms/step, n_out {out['n_out']}")
    cpu, parity = None, {"n_out": runs["full"]["n_out"], "l2": hex(runs["full"]["l2"]),
                         "modes_agree": all(runs[m]["n_out"] == runs["full"]["n_out"] and runs[m]["l2"] == runs["full"]["l2"]
                                            for m in runs)}
    if not args.no_cpu and os.path.exists(REF_DRIVER) and has_avx512():
        base = [REF_DRIVER, "pipeline", args.pipe_table, str(args.pipe_block), str(args.pipe_joins), "1",
                str(args.pipe_lhs), str(args.pipe_rhs)]
        ref = {}
        for compact, count_only in ((0, 0), (0, 1), (2, 1)):
            p = subprocess.run(base + [str(compact), str(count_only)], capture_output=True, text=True, timeout=900)
            t = p.stdout.split()
            ref[(compact, count_only)] = (int(t[t.index("n_out") + 1]), int(t[t.index("l2") + 1]),
                                          float(t[t.index("seconds") + 1]))
        n_ref, l2_ref, _ = ref[(0, 0)]
        parity.update(expected_n_out=n_ref, l1_ok=n_ref == runs["full"]["n_out"], l2_ok=l2_ref == runs["full"]["l2"])
        secs = ref[(2, 1)][2]
        cpu = {"value": args.pipe_lhs / secs, "unit": "LHS tuples/s", "cores": 1, "kind": "reference",
               "sample": (f"the whole workload: the reference's ExecutePipeline/FlushPipelineCache over its "
                          f"own classes (compiled from its sources, oracle/_ref/ref_driver), one thread, "
                          f"fixed compactor: {secs:.2f} s; no compaction: {ref[(0, 1)][2]:.2f} s "
                          f"(main.cpp's timed region, result collection off)"),
               "no_compact_value": args.pipe_lhs / ref[(0, 1)][2], "cpu_model": cpu_model()}
    full, none = runs["full"], runs["none"]
    line = {
        "metric": "pipeline LHS tuples/s (main.cpp multi-join pipeline with chunk compaction)",
        "value": args.pipe_lhs / full["s_per_step"], "unit": "LHS tuples/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": full["s_per_step"] * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
        "data": "synthetic: main.cpp's own generator (mt19937(2), uniform_int_distribution<int>(0, rhs))",
        "config": {"workload": (f"main.cpp pipeline: {args.pipe_joins} {args.pipe_table} joins, "
                                f"{args.pipe_lhs} LHS / {args.pipe_rhs} RHS, cf 1, B {args.pipe_block}"),
                   "compaction": "NaiveCompactor (fixed) between joins", "parallelism": "dp1"},
        "no_compaction": {"ms_per_step": none["s_per_step"] * 1e3, "value": args.pipe_lhs / none["s_per_step"],
                          "joins": none.get("joins")},
        "dynamic_compaction": {"ms_per_step": runs["dynamic"]["s_per_step"] * 1e3,
                               "value": args.pipe_lhs / runs["dynamic"]["s_per_step"],
                               "note": "UCB-tuned per-join thresholds (host/ccj_tuner.h), last steps after warm-up",
                               "tuner": runs["dynamic"].get("tuner")},
        "joins": full.get("joins"),
        "cpu_baseline": cpu,
        "parity": parity,
    }
    print(json.dumps(line), flush=True)


class _StdoutToStderr:
    """Route fd 1 to stderr while RCCL creates its communicator (it prints a banner on stdout;
    the driver reads bench.py's stdout as one JSON line)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 without an outside launcher: run torch.distributed.run as a CHILD process (this
    process never touches the GPU: no exec after a GPU call), one rank per GPU, and forward rank 0's
    single JSON line to stdout; everything else the ranks print goes to stderr.  Exit status: the
    launcher's (non-zero if any rank failed), or 1 if no JSON line came back."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[launch] {' '.join(cmd)}")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    for line in p.stdout:
        t = line.strip()
        if t.startswith("{") and '"metric"' in t:
            try:
                lines.append(json.loads(t))
                continue
            except ValueError:
                pass
        sys.stderr.write(line)
    rc = p.wait()
    if lines:
        print(json.dumps(lines[-1]), flush=True)
    if rc == 0 and not lines:
        log("[launch] no JSON line from rank 0")
        rc = 1
    return rc


def main():
    args = parse()
    if args.workload == "pipeline":  # runs the C++ driver in child processes
        return bench_pipeline(args)
    if (args.gpus > 1 or args.sharded) and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args)  # before any GPU call in this process (--sharded: one rank too)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.same_device else int(os.environ.get("LOCAL_RANK", "0"))
    if args.same_device and args.backend == "nccl" and world > 1:
        log("--same-device needs --backend gloo (RCCL refuses two ranks on one GPU)")
        return 2
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    if args.ops_module:  # tests: the N > 1 step on CPU tensors with gloo (no GPU)
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        return bench_multi(args, world, rank, local, torch.device("cpu"), None, dist)
    torch.cuda.set_device(local)
    ccj.device_init(local)
    dist = None
    if world > 1 or args.sharded:
        import torch.distributed as dist
        with _StdoutToStderr():
            if world == 1:
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                os.environ.setdefault("MASTER_PORT", "29533")
                dist.init_process_group(args.backend, rank=0, world_size=1, device_id=torch.device("cuda", local))
            elif args.backend == "nccl":
                dist.init_process_group(args.backend, device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(args.backend)
            dist.barrier()  # creates the communicator (and its banner) now
    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(device=dev)

    if world > 1 or args.sharded:
        return bench_multi(args, world, rank, local, dev, stream, dist)
    line = bench_c3(args, dev, stream) if args.workload == "c3" else bench_single(args, dev, stream)
    if args.workload == "c2" and not (args.no_other_workloads and args.no_scaling_reference):
        # the headline stands on its own if a later workload takes the process down
        log("[c2 line] " + json.dumps(line))
    if args.workload == "c2" and not args.no_other_workloads:
        line["other_workloads"] = other_workloads(args, dev, stream)
    if args.workload == "c2" and not args.no_scaling_reference:
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        line["scaling_reference"] = same_shape_n1(args, verify=not args.no_verify)
    print(json.dumps(line), flush=True)


def same_shape_n1(args, verify=True, steps=None, warmup=None):
    """The multi-GPU protocol at N = 1 on the per-GPU shape of the N > 1 lines (C4: --n-build-per-gpu
    build keys, --n-probe probe keys): owner split (one owner) + local copy + local probe, run by
    `bench.py --sharded` in a child process (its own one-rank launcher; this process never execs).
    The N = 1 point of the 1 -> 8 curve is THIS value, not the C2 headline: the same
    work per GPU as every N > 1 line, so value_N / (N * value_1) is the weak-scaling efficiency."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--sharded", "--gpus", "1", "--no-cpu",
           "--steps", str(steps or min(args.steps, 10)), "--warmup", str(warmup if warmup is not None else min(args.warmup, 2)),
           "--n-build-per-gpu", str(args.n_build_per_gpu), "--n-probe", str(args.n_probe), "--chunk", str(args.chunk),
           "--batches", str(args.batches), "--scaling", "weak"]
    if args.group:
        cmd += ["--group", str(args.group)]
    if not verify:
        cmd.append("--no-verify")
    if args.lib != "product":
        cmd += ["--lib", args.lib]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "GROUP_WORLD_SIZE", "ROLE_WORLD_SIZE")}
    t0 = time.perf_counter()
    try:
        p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    except subprocess.TimeoutExpired:
        return {"error": "timed out (600 s)"}
    ln = None
    for t in p.stdout.splitlines():
        t = t.strip()
        if t.startswith("{") and '"metric"' in t:
            try:
                ln = json.loads(t)
            except ValueError:
                pass
    if p.returncode != 0 or ln is None:
        return {"error": f"rc {p.returncode}: {p.stderr[-400:]}"}
    par = ln.get("parity", {})
    return {"protocol": "bench.py --sharded at N = 1 (owner split, local copy of the own segment, local probe)",
            "config": ln.get("config"), "ms_per_step": ln["ms_per_step"], "value": ln["value"], "unit": ln["unit"],
            "steps": ln["steps"], "warmup": ln["warmup"], "partition_ms": ln.get("partition_ms"),
            "exchange_ms": ln.get("exchange_ms"), "local_probe_ms": ln.get("local_probe_ms"),
            "l1_ok": par.get("l1_ok"), "l2_ok": par.get("l2_ok"), "matches": par.get("matches"),
            "expected_matches": par.get("expected_matches"), "wall_s": time.perf_counter() - t0,
            "use": "the N = 1 point of the multi-GPU curve (same per-GPU work as every N > 1 line)"}


def other_workloads(args, dev, stream):
    """BASELINE configs[2] (C3) and configs[4] (C5) timed in the same run as the C2 headline, each
    on its own buffers after the C2 ones are freed: the driver's default bench.py line then carries
    all three single-GPU workloads, each with its L1 / L2 check against the exact
    membership answer, its roofline (traffic from its committed counter profile) and its phases."""
    import copy
    res = []
    for w in ("c3", "c5"):
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        a = copy.copy(args)
        # C3 keeps its CPU baseline (the reference's chaining loop on 2^26 keys of the same stream,
        # bench_c3); C5 has no reference counterpart (the reference gathers no payload columns)
        a.workload, a.path, a.no_cpu, a.no_other = w, "partitioned", args.no_cpu or w != "c3", True
        a.cpu_sample = min(args.cpu_sample, 1 << 28)
        a.steps, a.warmup = max(1, min(args.steps, 10)), min(args.warmup, 2)
        t0 = time.perf_counter()
        try:
            ln = bench_c3(a, dev, stream) if w == "c3" else bench_single(a, dev, stream)
        except Exception as e:  # the C2 headline above stands on its own; report the failure beside it
            res.append({"workload": w, "error": f"{type(e).__name__}: {e}"[:500]})
            continue
        keep = {"workload": ln["config"]["workload"], "value": ln["value"], "unit": ln["unit"],
                "ms_per_step": ln["ms_per_step"], "steps": a.steps, "warmup": a.warmup, "path": ln.get("path"),
                "roofline": ln["roofline"], "phases": ln.get("phases"), "parity": ln["parity"],
                "cpu_baseline": ln.get("cpu_baseline"), "wall_s": time.perf_counter() - t0}
        if "compaction_ms" in ln:
            keep["compaction_ms"] = ln["compaction_ms"]
        res.append(keep)
        log(f"[other] {w}: {ln['ms_per_step']:.2f} ms/step, parity {ln['parity']}")
        del ln
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return res


def bench_single(args, dev, stream):
    """C2 (or C5) on one GPU: the BASELINE metric's step, its parity checks, roofline and CPU
    baseline; returns the JSON line's dict."""
    world, rank = 1, 0
    n_build, n_probe, chunk = args.n_build, args.n_probe, args.chunk
    layout = ccj.LAYOUT_DEVICE if args.layout == "device" else ccj.LAYOUT_REFERENCE

    # ---- setup (untimed, as the reference builds before its timer: main.cpp:62-68 vs :92-94) ----
    t0 = time.perf_counter()
    c5 = args.workload == "c5"
    P = 8 if c5 else 0
    # the rank walk is in libccj_tuning.so only: timed beside the headline with --lib tuning
    rank_ab = args.path == "partitioned" and not c5 and not args.no_other and args.lib == "tuning"
    with torch.cuda.stream(stream):
        table = ccj.Table.reference(ccj.LP, n_build, 1, layout, stream=stream)
        if c5:  # C5 payload of build tuple t (key k): p_c = k*(c+1)+c, row-major [n_build, 8]
            bk = ccj.gen_reference_keys(0, n_build, n_build, 1, stream=stream)
            mult = torch.arange(1, P + 1, dtype=torch.int64, device=dev)
            pay = bk[:, None] * mult[None, :] + (mult[None, :] - 1)
            table.set_payload(pay.reshape(-1), P, stream=stream)
            del bk, pay
        keys = ccj.gen_uniform_keys(n_probe, SEED, n_build, first_row=rank * n_probe, stream=stream)
        out = part = out_p = out_o = ws_o = None
        every = not c5 and not args.no_other  # C2: every path (the headline and the ones timed beside it)
        if args.path == "chunk" or every:
            out = table.alloc_outputs(n_probe, chunk, rounds=True, payload_cols=P, pos=c5)
        if args.path == "ordered" or every:
            out_o = table.alloc_outputs(n_probe, chunk, rounds=True)
            ws_o = table.alloc_ordered(n_probe, chunk)
        if args.path == "partitioned" or every:
            if rank_ab:  # the rank walk (tuning build only) is timed beside the headline (A/B)
                table.build_rank_index(stream=stream)
            part = table.alloc_partitioned(n_probe, chunk)
            # C5: the match positions the payload gather reads are a caller-owned buffer, so no
            # allocation runs inside the timed step
            out_p = table.alloc_outputs(part["positions"], chunk, rounds=False, payload_cols=P, pos=c5)
    stream.synchronize()
    log(f"[setup] table {table.size} slots, max_rounds {table.max_rounds}, keys {n_probe}: "
        f"{time.perf_counter() - t0:.1f} s")

    # C2 (distinct build keys, one output slot per position): CCJ_PART_ROWS — out_sel receives each
    # match's original row, and the split writes every position's key and row straight into the
    # output columns (ccj.h), so the walk only compacts chunks with misses
    # C5 too (round 3): the walk then writes only each match's table position, at its output slot
    rows_mode = int(table.max_dup) <= 1 and (not c5 or table.size <= 1 << 31) and not args.no_rows

    def step(path=args.path):
        if path == "partitioned":  # no host check inside the timed region: status is read after it
            table.probe_partitioned(keys, chunk, out=out_p, part=part, stream=stream, retry=False, rows=rows_mode)
        elif path == "rank":  # the rank walk (CCJ_PART_RANK, opt-in: A/B beside the headline)
            table.probe_partitioned(keys, chunk, out=out_p, part=part, stream=stream, retry=False, rows=rows_mode,
                                    rank=True)
        elif path == "ordered":  # L3 through the partitioned layout (status read after the timing)
            table.probe_ordered(keys, chunk, out=out_o, ws=ws_o, stream=stream, retry=False)
        else:
            table.probe(keys, chunk, out=out, stream=stream)

    for _ in range(args.warmup):
        step()
    stream.synchronize()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    pev = [ccj.PhaseEvents() for _ in range(args.steps)]  # the reference's 4-phase schema, per step
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        pev[i].arm()
        step()
        evs[i][1].record(stream)
    stream.synchronize()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ccj.PhaseEvents.disarm()
    phases = phase_report(pev, args.path, c5)
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    ms_per_step = wall * 1e3 / args.steps
    total_tuples = n_probe * world
    value = total_tuples / (wall / args.steps)

    # ---- verification + work accounting (untimed) ----
    if args.path == "partitioned":
        status = int(out_p["status"].item())
        if status & ccj.FLAG_PART_OVERFLOW:
            raise SystemExit("bench: fixed-capacity partition overflowed on uniform keys")
        out_p["n_chunks"] = (part["positions"] + chunk - 1) // chunk
        if rows_mode:  # sel = the original row
            matches, l2 = ccj.result_checksum(out_p, 0, row_base=rank * n_probe, stream=stream)
        else:
            rm = part["row_map"].to(torch.int64) + rank * n_probe
            matches, l2 = ccj.result_checksum(out_p, chunk, row_map=rm, stream=stream)
            del rm
    else:
        res0 = out_o if args.path == "ordered" else out
        status = int(res0["status"].item())
        matches, l2 = ccj.result_checksum(res0, chunk, row_base=rank * n_probe, stream=stream)
    # the other paths, timed the same way (reported beside the headline)
    others = [] if c5 or args.no_other else [q for q in ("ordered", "chunk", "partitioned") if q != args.path]
    if rank_ab:
        others.append("rank")  # A/B: the rank walk on the same split, same run
    other_runs = {}
    for other in others:
        step(other)
        stream.synchronize()
        ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for a, b in ev2:
            a.record(stream)
            step(other)
            b.record(stream)
        stream.synchronize()
        o_ms = sum(a.elapsed_time(b) for a, b in ev2) / len(ev2)
        if other in ("partitioned", "rank"):
            out_p["n_chunks"] = (part["positions"] + chunk - 1) // chunk
            if rows_mode:
                om, ol2 = ccj.result_checksum(out_p, 0, row_base=rank * n_probe, stream=stream)
            else:
                rm = part["row_map"].to(torch.int64) + rank * n_probe
                om, ol2 = ccj.result_checksum(out_p, chunk, row_map=rm, stream=stream)
                del rm
            o_par = {"status_flags": int(out_p["status"].item()), "matches": om, "l2": hex(ol2)}
        else:
            res = out_o if other == "ordered" else out
            om, ol2 = ccj.result_checksum(res, chunk, row_base=rank * n_probe, stream=stream)
            o_par = {"status_flags": int(res["status"].item()), "matches": om, "l2": hex(ol2)}
        other_runs[other] = (o_ms, o_par)
    l3_same = None
    if out is not None and out_o is not None and "chunk" in (other_runs.keys() | {args.path}):
        # L3 at full size: the ordered route's whole output equals probe_chunks' (counts, rounds,
        # every Next's count, and the ordered (sel, payload) stream of every chunk)
        torch.cuda.synchronize()
        same = all(torch.equal(out_o[k], out[k]) for k in ("count", "rounds", "round_counts"))
        if same:
            valid = (torch.arange(out["cap"], device=dev)[None, :] < out["count"].to(torch.int64)[:, None]).reshape(-1)
            same = bool(torch.equal(out_o["sel"][valid], out["sel"][valid])) and \
                bool(torch.equal(out_o["payload"][valid], out["payload"][valid]))
            del valid
        l3_same = same
        if "ordered" in other_runs:
            other_runs["ordered"][1]["equals_chunk_path_l3"] = same
    examined, cost_matches, walked, windows = table.probe_cost_walk(keys, stream=stream)
    parity = {"status_flags": status, "matches": matches, "l2": hex(l2)}
    if args.path == "ordered" and l3_same is not None:
        parity["equals_chunk_path_l3"] = l3_same
    if c5:  # every gathered payload column holds the matched build tuple's p_c (key == payload)
        torch.cuda.current_stream().wait_stream(stream)
        res = out_p if args.path == "partitioned" else out
        nc = res["n_chunks"]
        cnt = res["count"][:nc].to(torch.int64)
        valid = torch.arange(res["cap"], device=dev)[None, :] < cnt[:, None]
        pk = res["payload"][:nc * res["cap"]].view(-1, res["cap"])
        parity["payload_cols_ok"] = all(
            bool(((res["payload_cols"][c][:nc * res["cap"]].view(-1, res["cap"]) == pk * (c + 1) + c) | ~valid).all())
            for c in range(P))
        del cnt, valid, pk

    if not args.no_verify:
        from oracle import oracle as O
        want_m, want_l2 = O.count_uniform(SEED, rank * n_probe, (rank + 1) * n_probe, n_build, n_build, 1,
                                          threads=args.cpu_threads)
        parity.update(expected_matches=want_m, l1_ok=(want_m == matches), l2_ok=(want_l2 == l2))
        for _, o_par in other_runs.values():
            o_par.update(l1_ok=(want_m == o_par["matches"]), l2_ok=(hex(want_l2) == o_par["l2"]))
    s_bar = examined / n_probe
    m_bar = matches / n_probe
    alg_bytes_per_tuple = 8 + 8 * s_bar + m_bar * (12 + 16 * P)  # +16 B per payload column
    alg_bytes = alg_bytes_per_tuple * n_probe
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    # what the headline path's walk actually examines: with distinct build keys a row ends at its
    # first match (ccj.h ccj_probe_partitioned), so its slot words are s_walk, not the reference's
    # s_bar; the 32-byte windows it reads are the transaction-level view of the same walk
    first_match = args.path == "partitioned" and int(table.max_dup) <= 1
    s_walk = (walked if first_match else examined) / n_probe
    walked_bytes_per_tuple = 8 + 8 * s_walk + m_bar * (12 + 16 * P)
    window_bytes_per_tuple = 8 + 32 * windows / n_probe + m_bar * (12 + 16 * P)
    achieved_walked = walked_bytes_per_tuple * n_probe / (kern_ms * 1e-3) / 1e9
    # DRAM bytes per step of THIS path's kernels, from tools/profile.sh + tools/prof_summary.py (null
    # unless the profile was taken on this build: profile_traffic)
    prof = profile_traffic(args.workload, args.path, n_probe, n_build)
    traffic, kernels_ms = prof["traffic"], prof["kernels_ms"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and not c5:  # the reference has no payload gather
        cpu = cpu_baseline(args)
    ceiling = None
    if dev.type == "cuda" and n_probe >= (1 << 26):  # untimed, after the step's buffers are in place
        ceiling = copy_ceiling(dev, stream)

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "probe tuples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (reference key generator build side; SplitMix64 uniform probe keys, seed 42)",
            "config": {"workload": ("C5: 1xMI355X wide-payload LP join, 64M build / 1B probe int64, 8 int64 payload "
                                    "columns gathered on match, chunk=2048") if c5 else
                       "C2: 1xMI355X linear-probe, 64M build / 1B probe int64 uniform keys, chunk=2048",
                       "table": "linear_probing", "layout": args.layout, "n_build": n_build,
                       "n_probe_per_gpu": n_probe, "chunk": chunk, "parallelism": f"dp{world}"},
            "hbm_gbs_algorithmic": achieved,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_profile": prof["profile"], "traffic_profile_tag": prof["profile_tag"],
                         "traffic_profile_csrc_hash": prof["profile_csrc_hash"],
                         "traffic_stale": prof["traffic_stale"],
                         # measured DRAM bytes (whole 128-B lines per random slot read) per second
                         "traffic_GBps": traffic / (kern_ms * 1e-3) / 1e9 if traffic else None,
                         "kernel": (("ccj_probe_partitioned, CCJ_PART_ROWS (slot_split_pipe writing keys + rows, "
                                     "probe_walk2<POS> writing each chunk's matches by payload slab, "
                                     + ccj.last_gather_kernel() + ")") if c5 and
                                    args.path == "partitioned" and rows_mode else
                                    ("ccj_probe_partitioned (slot_split_pipe + probe_win<3> with positions + "
                                     "gather_payload_cols<8>)") if c5 and args.path == "partitioned" else
                                    "probe_chunks<LP,2> + gather_payload_cols<8>" if c5 else PATH_KERNELS[args.path]),
                         "gather_kernel_run": ccj.last_gather_kernel() if c5 else None,
                         "kernel_ms": kern_ms, "rocprof_kernels_ms": kernels_ms,
                         "alg_bytes_per_tuple": alg_bytes_per_tuple, "s_bar": s_bar, "m_bar": m_bar,
                         # the same step on the bytes its walk reads: slot words through the first
                         # match (distinct keys), not through the run's end
                         "frac_walked": achieved_walked / HBM_PEAK_GBS, "achieved_walked": achieved_walked,
                         "alg_bytes_walked_per_tuple": walked_bytes_per_tuple, "s_walk": s_walk,
                         "walk": "first match" if first_match else "whole run",
                         "window_bytes_per_tuple": window_bytes_per_tuple,
                         "windows_per_tuple": windows / n_probe,
                         # the same achieved rate against the copy rate measured on this box
                         "frac_of_copy_ceiling": achieved / ceiling["GBps"] if ceiling else None,
                         "frac_walked_of_copy_ceiling": achieved_walked / ceiling["GBps"] if ceiling else None},
            "phases": phases,
            "hbm_copy_ceiling": ceiling,
            "cpu_baseline": cpu,
            "parity": parity,
            "path": args.path,
            "other_paths": [{
                "path": o, "ms_per_step": o_ms, "value": n_probe / (o_ms * 1e-3),
                "frac": alg_bytes / (o_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                "parity": "L3 (reference order)" if o not in ("partitioned", "rank") else "L1/L2",
                "kernel": PATH_KERNELS[o], "check": o_par} for o, (o_ms, o_par) in other_runs.items()],
        }
    return line


def bench_multi(args, world, rank, local, dev, stream, dist):
    """C4 (BASELINE configs[3]): each rank owns 1/N of a build side of 2^27 * N reference keys
    (owner = top log2(N) hash bits; 2^30 in total at N = 8) and probes 2^30 keys of its own (weak
    scaling; --scaling strong: 2^30 / N each); a step = batched owner partition + RCCL
    all-to-all of (key, u32 row) + local probe, pipelined on three streams (ccj_dist.ShardedProbe).
    The line reports, per step and for the slowest rank, the busy time of each of the three streams
    (partition, exchange, local probe) and the bytes this rank sends over xGMI."""
    import ccj_dist
    ops = None
    if args.ops_module:  # tests: CPU ops object (gloo), no HIP
        import importlib.util
        spec = importlib.util.spec_from_file_location("bench_ops", args.ops_module)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        ops = mod.make_ops(rank)
    n_build_total = args.n_build_per_gpu * world
    n_probe = args.n_probe if args.scaling == "weak" else args.n_probe // world
    chunk = args.chunk
    group = args.group or ccj_dist.GROUP
    t0 = time.perf_counter()
    # the local split leaves CUs to the exchange's RCCL kernels and the next owner splits (one-rank
    # rehearsal, profiles/r5_ab_part_share.log: 19.95 ms per step with the share, 20.8 without —
    # the owner splits' busy time 10.3 -> 13.5 ms — although the probe alone is 14.75 -> 12.9 ms)
    part_share = args.part_share != "off"
    if ops is None:
        with torch.cuda.stream(stream):
            cu_split = tuple(int(x) for x in args.cu_split.split(",")) if args.cu_split else None
            sp = ccj_dist.ShardedProbe(n_build_total, 1, n_probe, chunk, world, rank, batches=args.batches,
                                       group=group, keep_rows=True,
                                       ops=ccj_dist.DeviceOps(cu_split=cu_split, share=part_share))
            keys = ccj.gen_uniform_keys(n_probe, SEED, n_build_total, first_row=rank * n_probe, stream=stream)
    else:
        sp = ccj_dist.ShardedProbe(n_build_total, 1, n_probe, chunk, world, rank, batches=args.batches, ops=ops,
                                   group=group, keep_rows=True)
        keys = ops.probe_keys(SEED, rank * n_probe, n_probe, n_build_total)
    o = sp.ops
    o.synchronize()
    log(f"[rank {rank}] setup {time.perf_counter() - t0:.1f} s, local build {sp.n_build_local}, "
        f"{sp.batches} batches in groups of {sp.group}, segment capacity {sp.seg_cap}")
    if args.warmup:
        sp.run(keys, rank * n_probe, steps=args.warmup)
    o.synchronize()
    dist.barrier()
    o.synchronize()
    sp.reset_timing()
    exact_before = sp.exact_steps
    t0 = time.perf_counter()
    # the K steps are issued back to back (ShardedProbe.run): step s + 1's partitions and exchanges
    # overlap step s's last local probe, and the ranks agree on the status word once, at the end
    sp.run(keys, rank * n_probe, steps=args.steps, timing=True)
    o.synchronize()
    dist.barrier()
    wall = time.perf_counter() - t0
    tdev = dev if dev.type == "cuda" else torch.device("cpu")

    def slowest(x):  # MAX over ranks
        t = torch.tensor([float(x)], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    wall = slowest(wall)
    phase = sp.timing_ms(args.steps)  # per step: partition / exchange / local-probe stream busy time
    phase = {k: slowest(v) for k, v in phase.items()}
    probe_ms = phase["local_probe_ms"]
    # timed steps redone with the exact-size protocol (every rank takes the same branch: the status
    # word is all-reduced before it, so this count is the same on all ranks)
    exact_fallback = sp.exact_steps - exact_before
    # the timed steps moved keys only: the groups whose results are still held get their probe rows
    # from the senders' kept per-batch row buffers (untimed all-to-all), checked against the exact
    # answer over those batches of every rank (a key-only step must stay traceable)
    resolved = None
    if not exact_fallback:
        rm_, rl_, covered = sp.resolve_kept_groups()
        t = torch.tensor([rm_, rl_ - (1 << 64) if rl_ >= (1 << 63) else rl_], dtype=torch.int64, device=tdev)
        dist.all_reduce(t)
        resolved = {"batches": covered, "matches": int(t[0].item()), "l2": hex(int(t[1].item()) % (1 << 64))}
        if not args.no_verify and rank == 0:
            from oracle import oracle as O
            wm_, wl_ = 0, 0
            for src in range(world):
                for i in covered:
                    lo, n = sp._batch(i)
                    a, b = O.count_uniform(SEED, src * n_probe + lo, src * n_probe + lo + n, n_build_total,
                                           n_build_total, 1, threads=args.cpu_threads)
                    wm_, wl_ = wm_ + a, (wl_ + b) % (1 << 64)
            resolved.update(l1_ok=wm_ == resolved["matches"], l2_ok=hex(wl_) == resolved["l2"])
    # the local probe alone (untimed steps over): the run's last group re-probed with nothing else
    # on the device, the slowest rank's — its own time beside the busy time shared with the other
    # two streams (the local probe against the single-GPU probe of the same table)
    probe_alone = slowest(sp.probe_alone_ms()) if not exact_fallback else None
    # the same group on the whole grid: the local probe's kernels without the CU share
    probe_alone_full = (slowest(sp.probe_alone_ms(share=False)) if not exact_fallback and part_share and ops is None
                        else None)
    # verification (untimed): global L1 / L2 against the exact membership answer
    m, l2 = sp.step(keys, rank * n_probe, verify=True)
    examined, received = 0, 0
    for i in range(sp.batches):  # S-bar over every received batch of the step
        rk = sp.received_keys(i)
        e, _ = o.probe_cost(rk, stream)
        examined, received = examined + e, received + rk.numel()
    tot = torch.tensor([m, l2 - (1 << 64) if l2 >= (1 << 63) else l2, examined, received], dtype=torch.int64,
                       device=tdev)
    dist.all_reduce(tot)
    m_all, l2_all = int(tot[0].item()), int(tot[1].item()) % (1 << 64)
    s_bar = int(tot[2].item()) / max(int(tot[3].item()), 1)
    xgmi = sp.xgmi_bytes_per_step()
    parity = {"matches": m_all, "l2": hex(l2_all), "exact_size_fallback_steps": exact_fallback,
              "timed_step_rows_resolved": resolved}
    if not args.no_verify and rank == 0:
        from oracle import oracle as O
        want_m, want_l2 = O.count_uniform(SEED, 0, world * n_probe, n_build_total, n_build_total, 1,
                                          threads=args.cpu_threads)
        parity.update(expected_matches=want_m, l1_ok=want_m == m_all, l2_ok=want_l2 == l2_all)
    m_bar = m_all / (world * n_probe)
    alg = 8 + 8 * s_bar + 12 * m_bar
    rows_local = int(tot[3].item()) / world  # tuples each rank probes locally per step (mean)
    achieved = alg * rows_local / (probe_ms * 1e-3) / 1e9 if probe_ms > 0 else None
    if rank == 0:
        value = world * n_probe / (wall / args.steps)
        line = {
            "metric": METRIC, "value": value, "unit": "probe tuples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall * 1e3 / args.steps,
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (reference key generator build side; SplitMix64 uniform probe keys, seed 42)",
            "config": {"workload": f"C4: {world}xMI355X radix-partitioned LP join, {n_build_total} build / "
                                   f"{world * n_probe} probe int64, chunk=2048, RCCL all-to-all tuple shuffle",
                       "table": "linear_probing", "n_build_total": n_build_total, "n_probe_per_gpu": n_probe,
                       "chunk": chunk, "batches": sp.batches, "group": sp.group,
                       "steps_pipelined": "the K steps issued back to back, one status agreement after them",
                       "parallelism": f"dp{world} (owner-partitioned)"},
            # per step, slowest rank; the three streams overlap, so these are busy times, not a sum
            "partition_ms": phase["partition_ms"], "exchange_ms": phase["exchange_ms"],
            "local_probe_ms": probe_ms,
            "local_probe_alone_ms": probe_alone,
            "local_probe_alone_rows": sp.group * sp.slots,
            "local_split_share": ("3/4 of the CUs (room for the exchange and the next owner splits)" if part_share
                                  else "all CUs") if ops is None else None,
            "local_probe_alone_full_grid_ms": probe_alone_full,
            "exchange": ("key-only all-to-all in timed steps (8 B per tuple + segment counts); each sender keeps its "
                         "rows per batch, so the held groups' matches are resolved to global rows after timing "
                         "(parity.timed_step_rows_resolved)"),
            "xgmi_bytes_per_step": xgmi["sent_to_peers"], "xgmi_useful_bytes_per_step": xgmi["useful_to_peers"],
            "xgmi_GBps_per_rank": xgmi["sent_to_peers"] / (wall / args.steps) / 1e9,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": None,
                         "kernel": "ccj_probe_partitioned (local split + walk of received tuples, slowest rank)",
                         "kernel_ms": probe_ms, "alg_bytes_per_tuple": alg, "s_bar": s_bar, "m_bar": m_bar,
                         "s_bar_over": "every received batch of one step, all ranks"},
            "cpu_baseline": None,
            "parity": parity,
        }
    dist.destroy_process_group()
    if rank == 0:
        if world > 1 and ops is None and not args.no_n1_same_shape:
            # the N = 1 point of this line's curve: the same per-GPU shape through the same protocol
            # (a child process on this rank's GPU, after the other ranks are done with theirs)
            torch.cuda.synchronize()
            del sp, keys
            torch.cuda.empty_cache()
            a1 = argparse.Namespace(**vars(args))
            if args.scaling == "strong":
                a1.n_probe = n_probe  # per-GPU probe keys of this line
            ref = same_shape_n1(a1, verify=False)
            line["n1_same_shape"] = ref
            line["n1_same_shape_ms"] = ref.get("ms_per_step")
            if ref.get("value"):
                line["per_gpu_value_vs_n1_same_shape"] = value / world / ref["value"]
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    sys.exit(main() or 0)
