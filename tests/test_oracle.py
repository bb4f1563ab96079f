"""Pins the CPU oracle (our C restatement) against vectors produced by the reference itself.

Golden data: tests/golden/*.npz + known_answers.json, made by tests/golden/make_golden.py from
oracle/_ref/ref_driver (reference sources compiled from /root/reference).  Parity level L3
(ordered per-Next stream) on every trace case, both the round view and chaining's merged view.
"""
import numpy as np
import pytest

from helpers import (assert_trace_equal, known_answers, load_trace, ref_keys, trace_inputs,
                     views_from_rounds)
from oracle import oracle as O

KA = known_answers()


def test_murmurhash64_known_values():
    # hash_functions.h:8-16: h(0) = 0; constants checked against a direct restatement.
    assert O.murmurhash64(0) == 0
    M = 0xFFFFFFFFFFFFFFFF

    def h(x):
        x ^= x >> 32
        x = (x * 0xD6E8FEB86659FD93) & M
        x ^= x >> 32
        x = (x * 0xD6E8FEB86659FD93) & M
        x ^= x >> 32
        return x

    for x in [1, 2, 12345, 2**63 - 1, 2**64 - 1, 0xDEADBEEF]:
        assert O.murmurhash64(x) == h(x)


@pytest.mark.parametrize("n,cf", [(1, 1), (5, 3), (4096, 1), (4096, 4), (4096, 64), (1000, 7), (1000000, 5)])
def test_ref_generator_and_membership(n, cf):
    keys = ref_keys(n, cf)
    vals, cnt = np.unique(keys, return_counts=True)
    for v, c in zip(vals[:50], cnt[:50]):
        assert O.ref_multiplicity(int(v), n, cf) == c
    probe = np.arange(0, int(keys.max()) + 3)
    got = sum(O.ref_multiplicity(int(k), n, cf) for k in probe[:2000])
    want = int(np.isin(keys, probe[:2000]).sum())
    assert got == want


@pytest.mark.parametrize("name", sorted(KA["trace_cases"]))
def test_oracle_matches_reference_traces(name):
    entry = KA["trace_cases"][name]
    spec = entry["spec"]
    kind = O.LP if spec["kind"] == "lp" else O.CHAIN
    table = O.Table(kind, ref_keys(spec["n_build"], spec["cf"]))
    for view, info in entry["views"].items():
        trace = load_trace(name, view)
        keys, sel, counts = trace_inputs(spec, trace)
        out = table.probe(keys, spec["B"], sel=sel, counts=counts, cap_factor=spec["cf"], max_rounds=512)
        got = views_from_rounds(out["count"], out["sel"], out["payload"], out["rounds"], out["round_counts"],
                                out["cap"], out["max_rounds"], merged=(view == "merged"))
        assert_trace_equal(got, trace)
        assert int(out["count"].sum()) == info["matches"]


@pytest.mark.parametrize("name", sorted(KA["sum_cases"]))
def test_oracle_matches_reference_sums(name):
    """Every SURVEY §4 known answer, the C2-size one included (survey_lp_2048_64M_64M: a 2^26-key
    LP table of 2^28 slots, 2^26 mt19937_64 probes): matches, L2, the order-sensitive L3 fold and
    the SURVEY checksum of the oracle's output equal the reference's own."""
    entry = KA["sum_cases"][name]
    spec = entry["spec"]
    want = entry["variants"]["next"]
    kind = O.LP if spec["kind"] == "lp" else O.CHAIN
    table = O.Table(kind, ref_keys(spec["n_build"], spec["cf"]))
    if spec["gen"] == 1:
        keys = O.mt64_keys(spec["seed"], spec["n_probe"], spec["range"])  # the SURVEY §4 driver's stream
    else:
        keys = O.uniform_keys(spec["seed"], 0, spec["n_probe"], spec["range"])
    out = table.probe(keys, spec["B"], cap_factor=spec["cf"], max_rounds=512)
    m, l2, l3, chk = O.result_sums(out["count"], out["sel"], out["payload"], out["cap"], spec["B"])
    assert (m, l2, l3, chk) == (want["matches"], want["l2"], want["l3"], want["survey_chk"])
    # size-independent exact counter (membership oracle) agrees too
    if spec["gen"] == 0:
        assert O.count_uniform(spec["seed"], 0, spec["n_probe"], spec["range"], spec["n_build"],
                               spec["cf"]) == (want["matches"], want["l2"])


def test_count_uniform_micro_bench_shape():
    # simd_micro_bench.cpp:78-81 with kHitFreq 1: every probe key lies in [0, kRHSTuples) and the
    # table holds 0..kRHSTuples-1 once, so #tuples == #probes (134217728 for 2^27).
    m, _ = O.count_uniform(9, 0, 1 << 20, 128, 128, 1)
    assert m == 1 << 20


@pytest.mark.parametrize("B", [4, 8, 2048])
def test_compact_plan_properties(B):
    rng = np.random.default_rng(B)
    segs = rng.integers(0, B + 1, size=300).astype(np.uint32)
    segs[::17] = B  # full chunks bypass the cache (compactor.cpp:6)
    dest, occ = O.compact_plan(segs, B)
    # a permutation into ceil-packed chunks, every chunk full except possibly the last
    assert len(np.unique(dest)) == len(dest)
    assert (occ[:-1] == B).all() and 0 < occ[-1] <= B
    assert int(occ.sum()) == int(segs.sum())
    # full segments land in one output chunk each, in order
    start = np.concatenate([[0], np.cumsum(segs.astype(np.int64))[:-1]])
    for s in np.flatnonzero(segs == B):
        d = dest[start[s]:start[s] + B]
        assert d[0] % B == 0 and (np.diff(d.astype(np.int64)) == 1).all()


def closed_form_compaction(segs, B, threshold=0):
    """The prefix-sum form the device compactor uses (csrc/ccj_compact.hip header)."""
    segs = np.asarray(segs, np.int64)
    thr = B if threshold == 0 or threshold > B else threshold
    full = (segs != 0) & (segs >= thr)
    t = np.concatenate([[0], np.cumsum(np.where(full, 0, segs))[:-1]])
    F = np.concatenate([[0], np.cumsum(full)[:-1]])
    E = np.where(t == 0, 0, (t + B - 1) // B - 1)
    fullE = E[full]
    dest = []
    for s, c in enumerate(segs):
        for j in range(c):
            if full[s]:
                dest.append((E[s] + F[s]) * B + j)
            else:
                u = t[s] + j
                k = u // B
                dest.append((k + np.searchsorted(fullE, k, side="right")) * B + u % B)
    return np.array(dest, np.int64)


@pytest.mark.parametrize("B,seed", [(4, 0), (4, 1), (8, 2), (16, 3), (5, 4)])
@pytest.mark.parametrize("threshold", [0, 1, 2, 3])
def test_compaction_closed_form_equals_sequential(B, seed, threshold):
    rng = np.random.default_rng(seed)
    segs = rng.integers(0, B + 1, size=400)
    segs[rng.random(400) < 0.2] = B
    dest, occ = O.compact_plan(segs.astype(np.uint32), B, threshold)
    assert np.array_equal(closed_form_compaction(segs, B, threshold), dest.astype(np.int64))
    # every row kept once; pass-through chunks keep their count, compacted ones are full but the last
    assert len(np.unique(dest)) == len(dest) and int(occ.sum()) == int(segs.sum())
    if threshold == 1:  # compacts nothing: one output chunk per non-empty result
        assert np.array_equal(occ, segs[segs > 0])


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("joins,n,rhs,cf,B", [(3, 3000, 500, 3, 128), (2, 2000, 300, 1, 2048), (1, 500, 40, 4, 64)])
def test_oracle_pipeline_is_the_join(kind, joins, n, rhs, cf, B):
    """The oracle's join-by-join pipeline (helpers.oracle_pipeline) yields exactly the multi-way
    join: every LHS row appears prod_l multiplicity(col_l) times with payload_l = col_l, with or
    without compaction (the two modes differ only in order)."""
    from helpers import oracle_pipeline
    cols = [O.uniform_keys(7 + j, 0, n, rhs + 1) for j in range(joins)]
    tables = [O.Table(kind, O.ref_build_keys(rhs, cf)) for _ in range(joins)]
    mult = np.ones(n, np.int64)
    for c in cols:
        mult *= np.array([O.ref_multiplicity(int(k), rhs, cf) for k in c])
    res = {}
    for compact in (False, True):
        out = oracle_pipeline(tables, cols, B, compact, cap_factor=cf)
        assert len(out[0]) == int(mult.sum())
        for l in range(joins):
            np.testing.assert_array_equal(out[joins + l], out[l])
        res[compact] = sorted(zip(*[o.tolist() for o in out]))
    assert res[False] == res[True]
    want = sorted(tuple(int(c[i]) for c in cols) for i in range(n) for _ in range(int(mult[i])))
    assert [r[:joins] for r in res[False]] == want


@pytest.mark.parametrize("n_build,cf", [(1 << 16, 1), (100000, 3)])
def test_c3_stream(n_build, cf):
    """C3 probe stream (ccj_gen.h ccj_c3_key): ~10 % hits, Zipf-like skew over the build keys,
    misses never match; count_c3 is the exact membership answer."""
    n = 1 << 20
    keys = O.c3_keys(42, 5, 5 + n, n_build, cf)
    mult = np.array([O.ref_multiplicity(int(k), n_build, cf) for k in keys[:20000]])
    hit = keys < n_build
    assert 0.095 < hit.mean() < 0.105
    assert ((mult > 0) == hit[:20000]).all()  # a hit is a build key, a miss never is
    _, c = np.unique(keys[hit], return_counts=True)
    assert c.max() > 50 * np.median(c)  # skewed: the top rank is hit far more than a typical key
    m, l2 = O.count_c3(42, 5, 5 + n, n_build, cf)
    rows = np.arange(5, 5 + n, dtype=np.uint64)
    mm = np.where(hit, np.array([O.ref_multiplicity(int(k), n_build, cf) if h else 0
                                 for k, h in zip(keys, hit)]), 0)
    assert m == int(mm.sum())
    assert l2 == O.l2_sum(np.repeat(rows, mm), np.repeat(keys, mm))
