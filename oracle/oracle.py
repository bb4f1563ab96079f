"""ctypes/numpy front end of the CPU oracle (liboracle.so).  TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker (or the timed CPU baseline).  The product path (libccj.so and the host
facade) never imports it.  See ccj_oracle.h for the reference file:line each function restates
and for the probe output contract.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

LP, CHAIN = 0, 1


def build(force: bool = False) -> str:
    path = os.path.join(HERE, "liboracle.so")
    if force or not os.path.exists(path):
        subprocess.run(["make", "-C", HERE, "oracle"], check=True, capture_output=True)
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = C.CDLL(build())
        u64, i64p, u64p, u32p = C.c_uint64, C.POINTER(C.c_int64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)
        L = _LIB
        L.ccj_o_murmurhash64.restype = u64
        L.ccj_o_murmurhash64.argtypes = [u64]
        L.ccj_o_ref_build_keys.restype = u64
        L.ccj_o_ref_build_keys.argtypes = [u64, u64, i64p]
        L.ccj_o_ref_multiplicity.restype = u64
        L.ccj_o_ref_multiplicity.argtypes = [C.c_int64, u64, u64]
        L.ccj_o_lp_num_slots.restype = u64
        L.ccj_o_lp_num_slots.argtypes = [u64]
        L.ccj_o_lp_build.argtypes = [i64p, u64, i64p, u64]
        L.ccj_o_lp_build_rows.argtypes = [i64p, u64, i64p, u32p, u64]
        L.ccj_o_chain_build_rows.argtypes = [i64p, u64, u64, u64p, i64p, u32p]
        L.ccj_o_chain_num_buckets.restype = u64
        L.ccj_o_chain_num_buckets.argtypes = [u64]
        L.ccj_o_chain_build.argtypes = [i64p, u64, u64, u64p, i64p]
        L.ccj_o_probe.restype = C.c_int
        L.ccj_o_probe.argtypes = [C.c_int, i64p, u64p, u64, i64p, u32p, u32p, u64, C.c_uint32, u64,
                                  C.c_uint32, u32p, u32p, i64p, u32p, u32p, C.c_int, u32p]
        L.ccj_o_probe_totals.restype = u64
        L.ccj_o_probe_totals.argtypes = [C.c_int, i64p, u64p, u64, i64p, u64, C.c_uint32, u64, u64p, C.c_int]
        L.ccj_o_gen_uniform.argtypes = [u64, u64, u64, u64, i64p, C.c_int]
        L.ccj_o_count_uniform.restype = u64
        L.ccj_o_count_uniform.argtypes = [u64, u64, u64, u64, u64, u64, u64p, C.c_int]
        L.ccj_o_gen_c3.argtypes = [u64, u64, u64, u64, u64, C.c_uint32, i64p, C.c_int]
        L.ccj_o_count_c3.restype = u64
        L.ccj_o_count_c3.argtypes = [u64, u64, u64, u64, u64, C.c_uint32, u64p, C.c_int]
        L.ccj_o_compact_plan.restype = u64
        L.ccj_o_compact_plan.argtypes = [u32p, u64, C.c_uint32, u64p, u32p]
        L.ccj_o_compact_plan_threshold.restype = u64
        L.ccj_o_compact_plan_threshold.argtypes = [u32p, u64, C.c_uint32, C.c_uint32, u64p, u32p]
        L.ccj_o_gen_mt64.argtypes = [u64, u64, u64, i64p]
        L.ccj_o_result_sums.argtypes = [u32p, u32p, i64p, u64, u64, C.c_uint32, u64p]
    return _LIB


def _p(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


def murmurhash64(x: int) -> int:
    return lib().ccj_o_murmurhash64(x & 0xFFFFFFFFFFFFFFFF)


def ref_build_keys(n: int, cf: int) -> np.ndarray:
    out = np.empty(n, dtype=np.int64)
    lib().ccj_o_ref_build_keys(n, cf, _p(out, C.c_int64))
    return out


def ref_multiplicity(k: int, n: int, cf: int) -> int:
    return lib().ccj_o_ref_multiplicity(k, n, cf)


class Table:
    """A CPU-side table in the same layout the device uses (LP slots / chaining CSR)."""

    def __init__(self, kind: int, keys: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        self.kind = kind
        L = lib()
        if kind == LP:
            self.size = L.ccj_o_lp_num_slots(len(keys))
            self.table = np.empty(self.size, dtype=np.int64)
            self.rows = np.empty(self.size, dtype=np.uint32)  # slot -> build tuple (UINT32_MAX = empty)
            L.ccj_o_lp_build_rows(_p(keys, C.c_int64), len(keys), _p(self.table, C.c_int64),
                                  _p(self.rows, C.c_uint32), self.size)
            self.bucket_off = None
        else:
            self.size = L.ccj_o_chain_num_buckets(len(keys))
            self.bucket_off = np.empty(self.size + 1, dtype=np.uint64)
            self.table = np.empty(len(keys), dtype=np.int64)
            self.rows = np.empty(len(keys), dtype=np.uint32)  # chain index -> build tuple
            L.ccj_o_chain_build_rows(_p(keys, C.c_int64), len(keys), self.size, _p(self.bucket_off, C.c_uint64),
                                     _p(self.table, C.c_int64), _p(self.rows, C.c_uint32))

    def probe(self, keys, chunk, sel=None, counts=None, cap_factor=1, max_rounds=256, threads=0):
        """Returns dict(count, sel, payload, rounds, round_counts) per the ccj_oracle.h contract."""
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        n_rows = len(keys)
        n_chunks = (n_rows + chunk - 1) // chunk
        cap = chunk * cap_factor
        out = dict(
            count=np.zeros(n_chunks, np.uint32),
            sel=np.zeros(n_chunks * cap, np.uint32),
            payload=np.zeros(n_chunks * cap, np.int64),
            rounds=np.zeros(n_chunks, np.uint32),
            round_counts=np.zeros(n_chunks * max_rounds, np.uint32),
            pos=np.zeros(n_chunks * cap, np.uint32),
        )
        if sel is not None:
            sel = np.ascontiguousarray(sel, dtype=np.uint32)
        if counts is not None:
            counts = np.ascontiguousarray(counts, dtype=np.uint32)
        rc = lib().ccj_o_probe(self.kind, _p(self.table, C.c_int64), _p(self.bucket_off, C.c_uint64), self.size,
                               _p(keys, C.c_int64), _p(sel, C.c_uint32), _p(counts, C.c_uint32), n_rows, chunk, cap,
                               max_rounds, _p(out["count"], C.c_uint32), _p(out["sel"], C.c_uint32),
                               _p(out["payload"], C.c_int64), _p(out["rounds"], C.c_uint32),
                               _p(out["round_counts"], C.c_uint32), threads, _p(out["pos"], C.c_uint32))
        if rc != 0:
            raise RuntimeError("oracle probe: output bound exceeded (cap_factor / max_rounds too small)")
        out["cap"] = cap
        out["max_rounds"] = max_rounds
        return out

    def probe_totals(self, keys, chunk, row_base=0, threads=0):
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        l2 = C.c_uint64(0)
        m = lib().ccj_o_probe_totals(self.kind, _p(self.table, C.c_int64), _p(self.bucket_off, C.c_uint64),
                                     self.size, _p(keys, C.c_int64), len(keys), chunk, row_base, C.byref(l2),
                                     threads)
        return int(m), int(l2.value)


def count_uniform(seed, row_begin, row_end, rng, n_build, cf, threads=0):
    l2 = C.c_uint64(0)
    m = lib().ccj_o_count_uniform(seed, row_begin, row_end, rng, n_build, cf, C.byref(l2), threads)
    return int(m), int(l2.value)


def c3_keys(seed, begin, end, n_build, cf, hit_ppm=100000, threads=0):
    """C3 probe keys of rows [begin, end) (ccj_gen.h ccj_c3_key)."""
    out = np.empty(end - begin, dtype=np.int64)
    lib().ccj_o_gen_c3(seed, begin, end - begin, n_build, cf, hit_ppm, _p(out, C.c_int64), threads)
    return out


def mt64_keys(seed, n, rng):
    """The SURVEY §4 driver's probe keys: mt19937_64(seed) % rng (ccj_o_gen_mt64)."""
    out = np.empty(n, dtype=np.int64)
    lib().ccj_o_gen_mt64(seed, n, rng, _p(out, C.c_int64))
    return out


def result_sums(count, sel, payload, cap, chunk):
    """(matches, L2, L3, SURVEY chk) of a probe output in stored order — the reference driver's
    sink (oracle/ref_driver.cpp Sink::Emit), so they compare directly with known_answers.json."""
    count = np.ascontiguousarray(count).view(np.uint32)
    sel = np.ascontiguousarray(sel).view(np.uint32)
    payload = np.ascontiguousarray(payload, dtype=np.int64)
    out = np.zeros(4, np.uint64)
    lib().ccj_o_result_sums(_p(count, C.c_uint32), _p(sel, C.c_uint32), _p(payload, C.c_int64), len(count), cap,
                            chunk, _p(out, C.c_uint64))
    return tuple(int(x) for x in out)


def count_c3(seed, begin, end, n_build, cf, hit_ppm=100000, threads=0):
    l2 = C.c_uint64(0)
    m = lib().ccj_o_count_c3(seed, begin, end, n_build, cf, hit_ppm, C.byref(l2), threads)
    return int(m), int(l2.value)


def compact_plan(seg_counts, chunk, threshold=0):
    """Literal sequential NaiveCompactor (fixed) over Next results of seg_counts rows: destination
    slot (out_chunk * chunk + offset) of every row, and the output chunks' row counts."""
    seg = np.ascontiguousarray(seg_counts, dtype=np.uint32)
    total = int(seg.sum())
    dest = np.zeros(total, np.uint64)
    occ = np.zeros(total // max(chunk, 1) + len(seg) + 2, np.uint32)
    n = lib().ccj_o_compact_plan_threshold(_p(seg, C.c_uint32), len(seg), chunk, threshold, _p(dest, C.c_uint64),
                                           _p(occ, C.c_uint32))
    return dest, occ[:n]


# ---- checksums (ccj_gen.h), vectorised ----
_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def fmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_keys(seed, begin, end, rng, threads=0):
    """SplitMix64 probe keys of rows [begin, end) (ccj_gen.h ccj_uniform_key)."""
    out = np.empty(end - begin, dtype=np.int64)
    lib().ccj_o_gen_uniform(seed, begin, end - begin, rng, _p(out, C.c_int64), threads)
    return out


def l2_sum(rows, payload) -> int:
    rows = np.asarray(rows, dtype=np.uint64)
    p = np.asarray(payload, dtype=np.int64).view(np.uint64)
    with np.errstate(over="ignore"):
        t = fmix64(rows * np.uint64(0x9E3779B97F4A7C15) + fmix64(p + np.uint64(1)))
        return int(np.sum(t, dtype=np.uint64))


def l3_fold(rows, payload, h=0x243F6A8885A308D3) -> int:
    h = np.uint64(h)
    for r, p in zip(np.asarray(rows, np.uint64), np.asarray(payload, np.int64).view(np.uint64)):
        h = fmix64(fmix64(h ^ r) ^ p)
    return int(h)
