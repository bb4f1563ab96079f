"""The device multi-join pipeline (ccj_pipeline_run, include/ccj.h) against
(1) the oracle's join-by-join restatement of main.cpp's ExecutePipeline (tests/helpers.py
oracle_pipeline) — the whole result table, in order (L3), with and without compaction — and
(2) the reference's own pipeline answers (tests/golden/known_answers.json pipe_cases) through the
C++ driver's batched engine (host/pipeline_main.cpp --engine batched): count, order-insensitive
checksum over every column, first result rows; plus the batched engine's full result order vs
the per-chunk facade running the reference's recursion (--dump)."""
import filecmp
import os
import subprocess

import numpy as np
import pytest

from helpers import known_answers, oracle_pipeline

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd", "host", "ccj_pipeline")
KA = known_answers()["pipe_cases"]
CASES = [k for k in sorted(KA) if "naive_compact" not in k and "16M" not in k]

pytestmark = pytest.mark.gpu


def _dev():
    import torch
    import ccj
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)
    return torch.device("cuda", 0)


def _inputs(joins, n, rhs, seed):
    from oracle import oracle as O
    return [O.uniform_keys(seed + j, 0, n, rhs + 1) for j in range(joins)]


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("compact", [False, True])
@pytest.mark.parametrize("joins,n,rhs,cf,B", [(3, 20000, 4000, 3, 256), (2, 5000, 1000, 1, 2048),
                                              (3, 3000, 200, 5, 64), (1, 777, 50, 2, 100), (4, 4096, 1500, 2, 512)])
def test_pipeline_l3_vs_oracle(kind, compact, joins, n, rhs, cf, B):
    import torch
    import ccj
    from oracle import oracle as O
    dev = _dev()
    cols = _inputs(joins, n, rhs, 11)
    dt = [ccj.Table.reference(kind, rhs, cf, ccj.LAYOUT_REFERENCE) for _ in range(joins)]
    ot = [O.Table(kind, O.ref_build_keys(rhs, cf)) for _ in range(joins)]
    want = oracle_pipeline(ot, cols, B, compact, cap_factor=cf)
    pl = ccj.Pipeline(dt, B, compact)
    pl.run([torch.from_numpy(c).to(dev) for c in cols])
    got = pl.result_columns()
    got = got[:joins] + [got[joins + 2 * l + 1] for l in range(joins)]
    assert pl.res.n_out == len(want[0])
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    st = pl.stats()
    assert st[0]["rows_in"] == n and st[-1]["rows_out"] == len(want[0])
    # the multiset does not depend on compaction; compaction never adds chunks
    n_chk, l2 = pl.checksum()
    other = ccj.Pipeline(dt, B, not compact)
    other.run([torch.from_numpy(c).to(dev) for c in cols])
    assert other.checksum() == (n_chk, l2)
    full, none = (pl, other) if compact else (other, pl)
    assert all(f["chunks_in"] <= g["chunks_in"] for f, g in zip(full.stats(), none.stats()))


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("thresholds,B", [((1, 1, 1), 256), ((64, 128, 0), 256), ((200, 1, 100), 256),
                                          ((1000, 0, 2048), 2048)])
def test_pipeline_threshold_compaction_l3(kind, thresholds, B):
    """Threshold-gated compactors between joins (ccj_pipeline_set_thresholds): the whole result
    table in order against the oracle pipeline with the same thresholds, and the same multiset as
    no compaction."""
    import torch
    import ccj
    from oracle import oracle as O
    dev = _dev()
    joins, n, rhs, cf = 3, 20000, 4000, 2
    cols = _inputs(joins, n, rhs, 5)
    dt = [ccj.Table.reference(kind, rhs, cf, ccj.LAYOUT_REFERENCE) for _ in range(joins)]
    ot = [O.Table(kind, O.ref_build_keys(rhs, cf)) for _ in range(joins)]
    want = oracle_pipeline(ot, cols, B, True, cap_factor=cf, thresholds=thresholds)
    pl = ccj.Pipeline(dt, B, True)
    pl.set_thresholds(thresholds)
    pl.run([torch.from_numpy(c).to(dev) for c in cols])
    got = pl.result_columns()
    got = got[:joins] + [got[joins + 2 * l + 1] for l in range(joins)]
    assert pl.res.n_out == len(want[0])
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
    none = ccj.Pipeline(dt, B, False)
    none.run([torch.from_numpy(c).to(dev) for c in cols])
    assert none.checksum() == pl.checksum()
    assert all(s["ms"] > 0 for s in pl.stats())


def test_pipeline_empty_and_no_match():
    import torch
    import ccj
    dev = _dev()
    t = [ccj.Table.reference(1, 100, 1, ccj.LAYOUT_REFERENCE) for _ in range(2)]
    for compact in (False, True):
        pl = ccj.Pipeline(t, 256, compact)
        pl.run([torch.zeros(0, dtype=torch.int64, device=dev)] * 2)
        assert pl.res.n_out == 0
        pl.run([torch.full((1000,), 10**9, dtype=torch.int64, device=dev)] * 2)  # no key matches
        assert pl.res.n_out == 0 and pl.stats()[0]["rows_out"] == 0
        assert pl.checksum() == (0, 0)


def run_bin(spec, engine, dump=None, extra=()):
    args = [BIN, "--join-num", spec["joins"], "--chunk-factor", spec["cf"], "--lhs-size", spec["lhs"],
            "--rhs-size", spec["rhs"], "--table", spec["kind"], "--compact", "full" if spec["compact"] else "none",
            "--block-size", spec["B"], "--engine", engine] + list(extra)
    if dump:
        args += ["--dump", dump]
    return subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=600)


def parse(out):
    res, head = {}, []
    for line in out.splitlines():
        t = line.split()
        if t and t[0] == "PIPE":
            res = {t[i]: int(t[i + 1]) for i in range(1, len(t), 2)}
        elif t and t[0] == "ROW":
            head.append([int(x) for x in t[1:]])
    return res, head


@pytest.mark.parametrize("name", sorted(k for k in KA if "naive_compact" not in k))  # incl. C1's 16M cases
def test_batched_engine_matches_reference(name):
    want = KA[name]
    p = run_bin(want["spec"], "batched")
    assert p.returncode == 0, p.stderr
    res, head = parse(p.stdout)
    assert res["n_out"] == want["n_out"]
    assert res["l2"] == want["l2"]
    assert head == want["head"]


@pytest.mark.parametrize("name", [k for k in CASES if "200k" in k or "300k" in k])
def test_batched_engine_order_equals_facade(name, tmp_path):
    spec = KA[name]["spec"]
    a, b = str(tmp_path / "facade.bin"), str(tmp_path / "batched.bin")
    p = run_bin(spec, "facade", a)
    assert p.returncode == 0, p.stderr
    q = run_bin(spec, "batched", b)
    assert q.returncode == 0, q.stderr
    assert os.path.getsize(a) == KA[name]["n_out"] * 8 * 3 * spec["joins"]
    assert filecmp.cmp(a, b, shallow=False)


@pytest.mark.parametrize("name", [k for k in CASES if k.startswith("main_") and "_j3_" in k and "compact" not in k])
@pytest.mark.parametrize("mode", ["thresholds", "dynamic"])
def test_gated_and_dynamic_compaction_match_reference(name, mode):
    """Threshold-gated compaction (fixed per join) and the UCB-tuned dynamic compaction give the
    reference's result multiset (count + order-insensitive checksum over every column)."""
    spec = KA[name]["spec"]
    B = spec["B"]
    extra = (["--compact", "full", "--thresholds", f"{B // 8},1,{B}"] if mode == "thresholds"
             else ["--compact", "dynamic", "--repeat", "60"])
    p = run_bin(spec, "batched", extra=extra)
    assert p.returncode == 0, p.stderr
    res, _ = parse(p.stdout)
    assert (res["n_out"], res["l2"]) == (KA[name]["n_out"], KA[name]["l2"])
    if mode == "dynamic":
        assert p.stderr.count("TUNER join") == 3


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("compact", [False, True])
def test_pipeline_large_tables_ordered_route_l3(kind, compact):
    """Tables past L2 / the Infinity Cache (>= 2^22 slots or buckets): ccj_pipeline_run probes the
    first join and every compacted input through ccj_probe_ordered (split + L2-resident walk +
    unsplit + reference-order emit) when the input fills the split's segments.  The whole result
    table in order (L3) against the oracle pipeline, cf 2 (runs / chains of several keys), ragged
    last chunk."""
    import torch
    import ccj
    from oracle import oracle as O
    dev = _dev()
    joins, n, rhs, cf, B = 3, (1 << 22) + 777, (1 << 22) + 5, 2, 2048
    cols = _inputs(joins, n, rhs, 29)
    dt = [ccj.Table.reference(kind, rhs, cf, ccj.LAYOUT_REFERENCE) for _ in range(joins)]
    # the partitioned route applies, and the input fills its segments (the pipeline's gate)
    assert dt[0].alloc_ordered(n, B) is not None
    assert ccj.lib().ccj_probe_partitioned_positions(dt[0]._h, n, B) * 3 <= n * 4
    ot = [O.Table(kind, O.ref_build_keys(rhs, cf)) for _ in range(joins)]
    want = oracle_pipeline(ot, cols, B, compact, cap_factor=cf)
    pl = ccj.Pipeline(dt, B, compact)
    pl.run([torch.from_numpy(c).to(dev) for c in cols])
    got = pl.result_columns()
    got = got[:joins] + [got[joins + 2 * l + 1] for l in range(joins)]
    assert pl.res.n_out == len(want[0]) > 0
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
