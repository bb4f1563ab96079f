#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ from the REFERENCE implementation.

Runs oracle/_ref/ref_driver — our driver (oracle/ref_driver.cpp) linked against the reference's
own sources compiled where they lie under /root/reference (oracle/Makefile, target `ref`).  This
script only runs in the build container, where the reference tree exists; the fixtures it writes
are data (inputs + expected outputs) and are committed so the tests never need the reference.

  python tests/golden/make_golden.py          # rebuilds _ref/ref_driver if needed
  python tests/golden/make_golden.py phys     # only the trace_*_phys.npz files
  python tests/golden/make_golden.py sums A B # only sum cases A, B (merged into known_answers.json)

Outputs
  trace_<case>_<view>.npz   per-Next traces (every Next call: chunk, rc, result.sel, payload)
  trace_<case>_phys.npz     per variant, result column m+1 over every physical row after each Next
  known_answers.json        counts / checksums for larger runs and the main.cpp pipeline
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")

# name: (kind, B, n_build, cf, n_probe, range, seed, gen, selmode)
TRACE_CASES = {
    "lp_b2048_cf1_hit": ("lp", 2048, 4096, 1, 8192, 4096, 1, 0, 0),
    "lp_b2048_cf4_hit": ("lp", 2048, 4096, 4, 8192, 4096, 2, 0, 0),
    "lp_b2048_cf1_miss_filtered": ("lp", 2048, 4096, 1, 8192, 40960, 3, 0, 1),
    "lp_b256_ragged_reversed": ("lp", 256, 4096, 1, 1000, 4096, 4, 0, 2),
    "lp_tiny_build": ("lp", 256, 1, 1, 512, 2, 5, 0, 0),
    "lp_cf3_odd": ("lp", 256, 5, 3, 700, 6, 6, 0, 1),
    "lp_cf64_long_runs": ("lp", 2048, 4096, 64, 4096, 4096, 7, 0, 0),
    "chain_b2048_cf1_hit": ("chain", 2048, 4096, 1, 8192, 4096, 1, 0, 0),
    "chain_b2048_cf4_hit": ("chain", 2048, 4096, 4, 8192, 4096, 2, 0, 0),
    "chain_b2048_cf1_miss_filtered": ("chain", 2048, 4096, 1, 8192, 40960, 3, 0, 1),
    "chain_b256_ragged_reversed": ("chain", 256, 4096, 1, 1000, 4096, 4, 0, 2),
    "chain_tiny_build": ("chain", 256, 1, 1, 512, 2, 5, 0, 0),
    "chain_cf64_long_chains": ("chain", 2048, 4096, 64, 4096, 4096, 7, 0, 0),
}
VARIANTS = ["next", "inone", "simdnext", "simdinone"]

# SURVEY §4 driver table (mt19937_64(42), key = g() % range, identity sel) + a SplitMix64 run.
SUM_CASES = {
    "survey_lp_2048_1M_16M_r1M": ("lp", 2048, 1000000, 1, 16000000, 1000000, 42, 1, 0),
    "survey_lp_2048_1M_16M_r10M": ("lp", 2048, 1000000, 1, 16000000, 10000000, 42, 1, 0),
    "survey_lp_2048_1M_4M_cf4": ("lp", 2048, 1000000, 4, 4000000, 1000000, 42, 1, 0),
    "survey_lp_256_1M_4M": ("lp", 256, 1000000, 1, 4000000, 1000000, 42, 1, 0),
    "survey_chain_2048_1M_16M_r1M": ("chain", 2048, 1000000, 1, 16000000, 1000000, 42, 1, 0),
    "survey_chain_2048_1M_16M_r10M": ("chain", 2048, 1000000, 1, 16000000, 10000000, 42, 1, 0),
    "survey_chain_2048_1M_4M_cf4": ("chain", 2048, 1000000, 4, 4000000, 1000000, 42, 1, 0),
    "survey_chain_256_1M_4M": ("chain", 256, 1000000, 1, 4000000, 1000000, 42, 1, 0),
    "splitmix_lp_2048_1M_4M_r3M_cf2": ("lp", 2048, 1000000, 2, 4000000, 3000000, 42, 0, 0),
    "splitmix_chain_2048_1M_4M_r3M_cf2": ("chain", 2048, 1000000, 2, 4000000, 3000000, 42, 0, 0),
    "survey_lp_2048_64M_64M": ("lp", 2048, 67108864, 1, 67108864, 67108864, 42, 1, 0),
    # chaining tables of 2^23 buckets (2^21 + 1 keys): large enough for ccj_probe_ordered's
    # partitioned route (>= 2^22 buckets), so the reference's chain vectors reach it
    "survey_chain_2048_2M_8M_r2M": ("chain", 2048, 2097153, 1, 8000000, 2097153, 42, 1, 0),
    "survey_chain_2048_2M_8M_r20M": ("chain", 2048, 2097153, 1, 8000000, 20971530, 42, 1, 0),
    "survey_chain_256_2M_4M_cf3": ("chain", 256, 2097153, 3, 4000000, 2097153, 42, 1, 0),
    "splitmix_chain_1000_2M_4M_r6M_cf2": ("chain", 1000, 2097153, 2, 4000000, 6000000, 42, 0, 0),
}

# main.cpp-shaped pipeline: (kind, B, joins, cf, lhs, rhs, compact)
PIPE_CASES = {
    "main_chain_j3_cf1_200k_20k": ("chain", 256, 3, 1, 200000, 20000, 0),
    "main_chain_j3_cf5_200k_20k": ("chain", 256, 3, 5, 200000, 20000, 0),
    "main_chain_j3_cf5_200k_20k_naive_compact": ("chain", 256, 3, 5, 200000, 20000, 1),
    "main_chain_j3_cf5_200k_20k_fixed_compact": ("chain", 256, 3, 5, 200000, 20000, 2),
    "main_chain_j3_cf1_200k_20k_fixed_compact": ("chain", 256, 3, 1, 200000, 20000, 2),
    "main_lp_j3_cf5_200k_20k": ("lp", 256, 3, 5, 200000, 20000, 0),
    "main_lp_j3_cf5_200k_20k_fixed_compact": ("lp", 256, 3, 5, 200000, 20000, 2),
    "main_chain_j1_cf1_16M_1M": ("chain", 256, 1, 1, 16000000, 1000000, 0),
    "main_lp_j1_cf1_16M_1M": ("lp", 256, 1, 1, 16000000, 1000000, 0),
    "main_chain_j3_cf2_2M_200k": ("chain", 256, 3, 2, 2000000, 200000, 0),
    "main_lp_j3_cf2_2M_200k": ("lp", 256, 3, 2, 2000000, 200000, 0),
    "main_chain_j2_cf3_300k_50k_b2048_fixed_compact": ("chain", 2048, 2, 3, 300000, 50000, 2),
    "main_chain_j2_cf3_300k_50k_b2048": ("chain", 2048, 2, 3, 300000, 50000, 0),
}


def run(args):
    return subprocess.run([DRIVER] + [str(a) for a in args], check=True, capture_output=True, text=True).stdout


def parse_sum(out):
    for line in out.splitlines():
        if line.startswith("SUM"):
            t = line.split()
            return {t[i]: int(t[i + 1]) for i in range(1, len(t), 2)}
    raise RuntimeError("no SUM line")


def parse_trace(out):
    chunk_counts, chunk_sel = [], []
    n_chunk, n_round, n_rc, m_sel, m_pay = [], [], [], [], []
    for line in out.splitlines():
        t = line.split()
        if t[0] == "C":
            chunk_counts.append(int(t[2]))
            chunk_sel.extend(int(x) for x in t[3:])
        elif t[0] == "N":
            n_chunk.append(int(t[1]))
            n_round.append(int(t[2]))
            n_rc.append(int(t[3]))
            for x in t[4:]:
                s, p = x.split(":")
                m_sel.append(int(s))
                m_pay.append(int(p))
    return dict(
        chunk_counts=np.array(chunk_counts, np.uint32),
        chunk_sel=np.array(chunk_sel, np.uint32),
        next_chunk=np.array(n_chunk, np.uint32),
        next_round=np.array(n_round, np.uint32),
        next_rc=np.array(n_rc, np.uint32),
        match_sel=np.array(m_sel, np.uint32),
        match_payload=np.array(m_pay, np.int64),
    )


def parse_phys(out):
    """Per Next call: the fold of result column m+1 over all kBlockSize physical rows ("P" lines)."""
    return np.array([int(l.split()[1]) for l in out.splitlines() if l.startswith("P ")], np.uint64)


def make_phys():
    """trace_<case>_phys.npz: per variant, the physical payload-column fold after every Next call.
    Next / SIMDNext write matched rows only; InOneNext / SIMDInOneNext also write the visited value of
    every unmatched active row (linear_probing_ht.cpp:133, chaining_ht.cpp:156)."""
    for name, (kind, B, n, cf, npb, rng, seed, gen, selm) in TRACE_CASES.items():
        ph = {v: parse_phys(run(["probe", kind, v, B, n, cf, npb, rng, seed, gen, selm, 1])) for v in VARIANTS}
        assert np.array_equal(ph["next"], ph["simdnext"]) and np.array_equal(ph["inone"], ph["simdinone"]), name
        np.savez_compressed(os.path.join(HERE, f"trace_{name}_phys.npz"), **ph)
        print("phys", name, {v: len(x) for v, x in ph.items()}, flush=True)


def sum_case(name):
    kind, B, n, cf, npb, rng, seed, gen, selm = SUM_CASES[name]
    vs = ["next", "simdinone"] if n > 10_000_000 else VARIANTS
    res = {}
    for v in vs:
        res[v] = parse_sum(run(["probe", kind, v, B, n, cf, npb, rng, seed, gen, selm, 0]))
    for v in vs[1:]:
        for k in ("matches", "l2", "survey_chk"):
            assert res[v][k] == res[vs[0]][k], (name, v, k)
    print("sum", name, res[vs[0]]["matches"], hex(res[vs[0]]["survey_chk"]), flush=True)
    return {"spec": dict(kind=kind, B=B, n_build=n, cf=cf, n_probe=npb, range=rng, seed=seed, gen=gen,
                         selmode=selm), "variants": res}


def same(a, b):
    return all(np.array_equal(a[k], b[k]) for k in a)


def main():
    if not os.path.exists(DRIVER):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    if sys.argv[1:2] == ["sums"]:  # add / refresh only the named sum cases
        path = os.path.join(HERE, "known_answers.json")
        with open(path) as f:
            answers = json.load(f)
        for name in sys.argv[2:]:
            answers["sum_cases"][name] = sum_case(name)
        with open(path, "w") as f:
            json.dump(answers, f, indent=1, sort_keys=True)
        return 0
    make_phys()
    if sys.argv[1:] == ["phys"]:
        return 0
    answers = {"trace_cases": {}, "sum_cases": {}, "pipe_cases": {}}
    for name, (kind, B, n, cf, npb, rng, seed, gen, selm) in TRACE_CASES.items():
        traces = {}
        for v in VARIANTS:
            out = run(["probe", kind, v, B, n, cf, npb, rng, seed, gen, selm, 1])
            traces[v] = (parse_trace(out), parse_sum(out))
        # Views: "rounds" = one Next per probe round (LP: every variant; chaining: InOneNext forms,
        # chaining_ht.cpp:138-173); "merged" = chaining Next/SIMDNext, whose ScanInnerJoin repeats
        # rounds until >= 1 match (chaining_ht.cpp:82-107).
        views = {"rounds": ["next", "inone", "simdnext", "simdinone"]} if kind == "lp" else {
            "rounds": ["inone", "simdinone"], "merged": ["next", "simdnext"]}
        entry = {"spec": dict(kind=kind, B=B, n_build=n, cf=cf, n_probe=npb, range=rng, seed=seed, gen=gen,
                              selmode=selm), "views": {}}
        for view, vs in views.items():
            t0, s0 = traces[vs[0]]
            for v in vs[1:]:
                assert same(t0, traces[v][0]), f"{name}: variant {v} disagrees with {vs[0]}"
                assert s0 == traces[v][1]
            np.savez_compressed(os.path.join(HERE, f"trace_{name}_{view}.npz"), **t0)
            entry["views"][view] = {"variants": vs, **s0}
        answers["trace_cases"][name] = entry
        print("trace", name, {v: e["matches"] for v, e in entry["views"].items()}, flush=True)
    for name in SUM_CASES:
        answers["sum_cases"][name] = sum_case(name)
    for name, (kind, B, joins, cf, lhs, rhs, compact) in PIPE_CASES.items():
        out = run(["pipeline", kind, B, joins, cf, lhs, rhs, compact])
        head = []
        res = {}
        for line in out.splitlines():
            t = line.split()
            if t[0] == "PIPE":
                res = {t[i]: int(t[i + 1]) for i in range(1, len(t), 2)}
            elif t[0] == "ROW":
                head.append([int(x) for x in t[1:]])
        answers["pipe_cases"][name] = {"spec": dict(kind=kind, B=B, joins=joins, cf=cf, lhs=lhs, rhs=rhs,
                                                    compact=compact), **res, "head": head}
        print("pipe", name, res["n_out"], flush=True)
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(answers, f, indent=1, sort_keys=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
