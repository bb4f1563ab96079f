"""Seeded random sweep over the probe entry points, each case checked against the oracle.

Each case draws its configuration from its seed:
  - table kind (LP / chaining);
  - build keys: distinct, or with duplicates, some negative;
  - probe keys: hits, misses, a hot key (skew), empty markers (-1) and other negative keys;
  - chunk width from 1 to 2048, and a ragged last chunk.
Every entry point that takes the configuration is run on it, through the C ABI:
  ccj_probe              L3: every Next's rows in round-major order equal the oracle's
                         (oracle/ccj_oracle.c, after linear_probing_ht.cpp:62-115 /
                         chaining_ht.cpp:82-107), in the rounds view and the merged view
  ccj_probe_ordered      L3: the same comparison
  ccj_compact            the chunk path's Next results re-chunked: every row's output slot, the
                         output chunk counts and the carried columns equal the oracle's sequential
                         compactor on the oracle's Next results (threshold and key-column options drawn)
  ccj_probe_partitioned  L1 + L2: the multiset of (probe row, payload) equals the oracle's
  device-built tables    the same keys built by ccj_table_build_on_device: chaining (byte-identical
                         to the host build) at L3, LP (atomicCAS placement) at L1 + L2
  LP, distinct keys:     rows mode (CCJ_PART_ROWS) gives the same multiset; with 8 payload columns
                         and match positions, on both the chunk path (L3: positions equal the
                         oracle's) and the partitioned path (slab order where it applies), every
                         gathered column is the matched build tuple's.
  filtered input         a drawn selection vector and per-chunk counts (the pipeline's chunk form):
                         the chunk path at L3 against the oracle on the same sel / counts
  ccj_pipeline_run       1-4 joins of drawn tables and columns, no compaction / NaiveCompactor /
                         drawn thresholds, against the oracle's join-by-join restatement of
                         main.cpp:119-191 (tests/helpers.py oracle_pipeline): the result table in order
The cases complement the fixed-shape tests: shapes nobody picked by hand."""
import os

import numpy as np
import pytest

from helpers import assert_trace_equal, oracle_pipeline, views_from_rounds
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

# 64 fixed cases by default; CCJ_SWEEP_CASES / CCJ_SWEEP_BASE run a longer exploratory sweep
N_CASES = int(os.environ.get("CCJ_SWEEP_CASES", "64"))
BASE = int(os.environ.get("CCJ_SWEEP_BASE", "0"))
GATHERS = set()  # the gather kernels the partitioned payload probes ran (ccj_last_gather_kernel)
P = 8  # payload columns


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


def draw(case):
    """The case's configuration: (kind, build keys, probe keys, chunk)."""
    r = np.random.default_rng(7001 + BASE + case)
    kind = ccj.CHAIN if case % 3 == 2 else ccj.LP
    n_build = int(r.choice([1, 5, 300, 4096, 50000, 1 << 18, (1 << 20) + 17, 1 << 21]))
    distinct = bool(r.random() < 0.6)
    base = int(r.integers(0, 1 << 40))
    if distinct:
        bk = base + r.permutation(2 * n_build)[:n_build].astype(np.int64)
    else:
        bk = base + r.integers(0, max(1, n_build // 3), n_build, dtype=np.int64)
    chunk = int(r.choice([1, 2, 63, 64, 100, 256, 1000, 1023, 2047, 2048, 2048, 2048]))
    n_probe = int(r.choice([1, 999, 1 << 16, 300001, 1 << 20, (1 << 22) - 5]))
    if not distinct or chunk < 64:
        n_probe = min(n_probe, 1 << 18)  # outputs of chunk * max_dup rows per chunk
    hit = float(r.random())
    keys = np.where(r.random(n_probe) < hit, bk[r.integers(0, n_build, n_probe)],
                    base + 2 * n_build + r.integers(0, 2 * n_build + 1, n_probe))
    if r.random() < 0.3:  # a hot key: one build key in ~1/5 of the rows
        keys[r.random(n_probe) < 0.2] = bk[0]
    if r.random() < 0.3:  # the empty marker and other negative keys never match
        keys[::101] = -1
        keys[50::103] = -(1 << 62)
    bk, keys = bk.astype(np.int64), keys.astype(np.int64)
    if np.random.default_rng(99 + BASE + case).random() < 0.25:
        # negative build keys, the same keys negated in both columns (never -1: the LP empty marker)
        bk = np.where((bk > 1) & (bk % 5 == 0), -bk, bk)
        keys = np.where((keys > 1) & (keys % 5 == 0), -keys, keys)
    return kind, bk, keys, chunk


def payload_rows(n):
    g = np.arange(n, dtype=np.uint64)[:, None] * np.uint64(P) + np.arange(P, dtype=np.uint64)[None, :]
    return O.fmix64(g).view(np.int64)


def host(o):
    torch.cuda.synchronize()

    def conv(v):
        if isinstance(v, torch.Tensor):
            return v.cpu().numpy()
        return [conv(x) for x in v] if isinstance(v, list) else v
    return {k: conv(v) for k, v in o.items()}


def valid_of(count, n_chunks, cap):
    cnt = np.asarray(count[:n_chunks]).view(np.uint32).astype(np.int64)
    return cnt, (np.arange(cap)[None, :] < cnt[:, None]).reshape(-1)


def pairs(rows, pay):
    rows = np.asarray(rows, np.int64)
    pay = np.asarray(pay, np.int64)
    o = np.lexsort((pay, rows))
    return rows[o], pay[o]


def assert_same_pairs(got, want, what):
    g, w = pairs(*got), pairs(*want)
    assert len(g[0]) == len(w[0]), (what, len(g[0]), len(w[0]))
    assert np.array_equal(g[0], w[0]) and np.array_equal(g[1], w[1]), what


def assert_l3(out, want, kind):
    for merged in ((False, True) if kind == ccj.CHAIN else (False,)):
        g = views_from_rounds(out["count"], out["sel"].view(np.uint32), out["payload"], out["rounds"],
                              out["round_counts"], out["cap"], out["max_rounds"], merged=merged)
        w = views_from_rounds(want["count"], want["sel"], want["payload"], want["rounds"], want["round_counts"],
                              want["cap"], want["max_rounds"], merged=merged)
        assert_trace_equal(g, w)


def check_compaction(case, out_d, want, keys, d_keys, chunk):
    """ccj_compact of the chunk path's Next results against the oracle's sequential NaiveCompactor
    (compact_plan: compactor.cpp:5-41, the :36 fix) run on the ORACLE's Next results: output chunk
    counts and every row's global row, payload and carried columns (DataChunk::Append, base.cpp:15-27),
    with the case's pass-through threshold and, for odd cases, the key column filled from the payload."""
    r = np.random.default_rng(9001 + BASE + case)
    threshold = int(r.choice([0, 1, max(1, chunk // 2), chunk]))
    extra = (np.arange(len(keys), dtype=np.int64) * 7 - 3)
    d_extra = torch.from_numpy(extra).cuda()
    key_cols = [0] if case % 2 else []
    comp = ccj.compact(out_d, chunk, cols=[d_keys, d_extra], threshold=threshold, key_cols=key_cols)
    torch.cuda.synchronize()
    assert int(comp["status"].item()) == 0
    cap, mr = want["cap"], want["max_rounds"]
    segs, rows, pays = [], [], []
    for c in range(len(want["count"])):
        k = int(want["count"][c])
        segs.extend(int(x) for x in want["round_counts"][c * mr:c * mr + int(want["rounds"][c])])
        rows.append(c * chunk + want["sel"][c * cap:c * cap + k].astype(np.int64))
        pays.append(want["payload"][c * cap:c * cap + k])
    rows = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    pays = np.concatenate(pays) if pays else np.zeros(0, np.int64)
    dest, occ = O.compact_plan(np.array(segs, np.uint32), chunk, threshold)
    dest = dest.astype(np.int64)
    n_out = int(comp["n"].item())
    assert n_out == len(occ)
    assert np.array_equal(comp["counts"].cpu().numpy()[:n_out].view(np.uint32), occ)
    lim = n_out * chunk
    assert np.array_equal(comp["row"].cpu().numpy()[:lim][dest], rows)
    assert np.array_equal(comp["payload"].cpu().numpy()[:lim][dest], pays)
    assert np.array_equal(comp["cols"][0].cpu().numpy()[:lim][dest], keys[rows])
    assert np.array_equal(comp["cols"][1].cpu().numpy()[:lim][dest], extra[rows])
    assert int(occ.sum()) == len(rows)  # nothing lost, nothing added


@pytest.mark.parametrize("case", range(N_CASES))
def test_sweep_case(case):
    kind, bk, keys, chunk = draw(case)
    n = len(keys)
    table = ccj.Table.from_host(kind, bk)
    otab = O.Table(kind, bk)
    dup = max(1, int(table.max_dup))
    d_keys = torch.from_numpy(keys).cuda()

    # L3: the chunk path and the ordered path, against the oracle
    out_d = table.probe(d_keys, chunk)
    out = host(out_d)
    assert out["status"][0] == 0, hex(int(out["status"][0]))
    want = otab.probe(keys, chunk, cap_factor=dup, max_rounds=out["max_rounds"])
    assert_l3(out, want, kind)
    check_compaction(case, out_d, want, keys, d_keys, chunk)
    ordered = host(table.probe_ordered(d_keys, chunk))
    assert ordered["status"][0] == 0, hex(int(ordered["status"][0]))
    assert_l3(ordered, want, kind)

    # the oracle's matches as (probe row, payload)
    n_chunks = (n + chunk - 1) // chunk
    wcnt, wvalid = valid_of(want["count"], n_chunks, want["cap"])
    wrow = np.repeat(np.arange(n_chunks, dtype=np.int64), wcnt) * chunk + want["sel"][wvalid].astype(np.int64)
    wpay = want["payload"][wvalid]
    wpos = want["pos"][wvalid]

    # the device build of the same keys (ccj_table_build_on_device): chaining is byte-identical to
    # the host build, so L3 holds; the LP device build places keys by atomicCAS: L1 + L2
    dt = ccj.Table.on_device(kind, torch.from_numpy(bk).cuda())
    assert int(dt.max_dup) == dup
    h = host(dt.probe(d_keys, chunk))
    assert h["status"][0] == 0, hex(int(h["status"][0]))
    if kind == ccj.CHAIN:
        assert_l3(h, want, kind)
    else:
        cnt, valid = valid_of(h["count"], n_chunks, h["cap"])
        grow = np.repeat(np.arange(n_chunks, dtype=np.int64), cnt) * chunk + h["sel"].view(np.uint32)[valid]
        assert_same_pairs((grow, h["payload"][valid]), (wrow, wpay), "device-built LP")
    dt.free()

    # L1 + L2: the partitioned probe (the row map takes a position back to its row)
    part = table.probe_partitioned(d_keys, chunk)
    h = host(part)
    assert h["status"][0] == 0, hex(int(h["status"][0]))
    cnt, valid = valid_of(h["count"], h["n_chunks"], h["cap"])
    gpos = np.repeat(np.arange(h["n_chunks"], dtype=np.int64), cnt) * chunk + \
        h["sel"].view(np.uint32)[:h["n_chunks"] * h["cap"]][valid].astype(np.int64)
    grow = h["row_map"].view(np.uint32)[gpos].astype(np.int64)
    assert_same_pairs((grow, h["payload"][:h["n_chunks"] * h["cap"]][valid]), (wrow, wpay), "partitioned")

    if kind != ccj.LP or dup != 1 or table.size < 16:
        table.free()
        return
    # LP, distinct keys (a table of >= 16 slots): rows mode
    h = host(table.probe_partitioned(d_keys, chunk, rows=True))
    assert h["status"][0] == 0, hex(int(h["status"][0]))
    cnt, valid = valid_of(h["count"], h["n_chunks"], h["cap"])
    grow = h["sel"].view(np.uint32)[:h["n_chunks"] * h["cap"]][valid].astype(np.int64)
    assert_same_pairs((grow, h["payload"][:h["n_chunks"] * h["cap"]][valid]), (wrow, wpay), "rows mode")
    # payload columns: the chunk path (positions at L3) and the partitioned path (slab order)
    pay = payload_rows(len(bk))
    table.set_payload(torch.from_numpy(pay.reshape(-1)).cuda(), P)
    h = host(table.probe(d_keys, chunk, pos=True, payload_cols=P))
    assert h["status"][0] == 0, hex(int(h["status"][0]))
    assert np.array_equal(h["count"].view(np.uint32), want["count"])
    _, valid = valid_of(h["count"], n_chunks, h["cap"])
    pos = h["pos"].view(np.uint32)[valid]
    assert np.array_equal(pos, wpos)
    for c in range(P):
        assert np.array_equal(h["payload_cols"][c][valid], pay[otab.rows[pos], c]), ("chunk path column", c)
    h = host(table.probe_partitioned(d_keys, chunk, rows=True, pos=True, payload_cols=P))
    GATHERS.add(ccj.last_gather_kernel().split("<")[0])
    assert h["status"][0] == 0, hex(int(h["status"][0]))
    cnt, valid = valid_of(h["count"], h["n_chunks"], h["cap"])
    lim = h["n_chunks"] * h["cap"]
    grow = h["sel"].view(np.uint32)[:lim][valid].astype(np.int64)
    gkey = h["payload"][:lim][valid]
    assert_same_pairs((grow, gkey), (wrow, wpay), "payload columns")
    pos = h["pos"].view(np.uint32)[:lim][valid]
    assert np.array_equal(otab.table[pos], gkey)  # the position holds the row's key
    for c in range(P):
        assert np.array_equal(h["payload_cols"][c][:lim][valid], pay[otab.rows[pos], c]), ("partitioned column", c)
    table.free()


def test_sweep_ran_both_gathers():
    """The sweep reached the slab-order gather and the per-chunk one (collected by the cases above;
    skipped when they were not run in this session)."""
    if not GATHERS:
        pytest.skip("needs test_sweep_case's payload cases in the same session")
    assert {"gather_payload_cols", "gather_payload_cols_sub"} <= GATHERS, GATHERS


def test_sweep_filtered_input():
    """Chunks with a selection vector and per-chunk counts (a chunk's rows are sel[c*B, c*B + counts[c]),
    in sel's order; linear_probing_ht.cpp:39-60 takes (join_key, count, sel)): L3 against the oracle."""
    for case in range(8):
        kind, bk, keys, chunk = draw(100 + case)
        r = np.random.default_rng(5001 + case)
        n_chunks = (len(keys) + chunk - 1) // chunk
        keys = np.concatenate([keys, np.full(n_chunks * chunk - len(keys), -1, np.int64)])  # whole chunks
        sel = np.concatenate([r.permutation(chunk) for _ in range(n_chunks)]).astype(np.uint32)
        counts = r.integers(0, chunk + 1, n_chunks).astype(np.uint32)
        table = ccj.Table.from_host(kind, bk)
        otab = O.Table(kind, bk)
        out = host(table.probe(torch.from_numpy(keys).cuda(), chunk, sel=torch.from_numpy(sel.view(np.int32)).cuda(),
                               counts=torch.from_numpy(counts.view(np.int32)).cuda()))
        assert out["status"][0] == 0, (case, hex(int(out["status"][0])))
        want = otab.probe(keys, chunk, sel=sel, counts=counts, cap_factor=max(1, int(table.max_dup)),
                          max_rounds=out["max_rounds"])
        assert_l3(out, want, kind)
        table.free()


def draw_pipeline(case):
    r = np.random.default_rng(8001 + BASE + case)
    joins = int(r.integers(1, 5))
    B = int(r.choice([1, 7, 64, 100, 256, 1000, 2048]))
    n = int(r.choice([1, 500, 5000, 20000]))
    if B < 64:
        n = min(n, 3000)
    tables, cols = [], []
    for _ in range(joins):
        kind = ccj.LP if r.random() < 0.5 else ccj.CHAIN
        nb = int(r.choice([1, 10, 300, 4000]))
        base = int(r.integers(0, 1 << 40))
        if r.random() < 0.5:
            bk = base + r.permutation(2 * nb)[:nb].astype(np.int64)
        else:
            bk = base + r.integers(0, max(1, nb // 2), nb, dtype=np.int64)
        hit = float(r.random())
        col = np.where(r.random(n) < hit, bk[r.integers(0, nb, n)], base + 2 * nb + r.integers(0, 100, n))
        tables.append((kind, bk.astype(np.int64)))
        cols.append(col.astype(np.int64))
    compact = bool(r.random() < 0.6)
    thresholds = [int(r.choice([0, 1, max(1, B // 2), B])) for _ in range(joins)] if compact and r.random() < 0.5 \
        else None
    return tables, cols, B, compact, thresholds


@pytest.mark.parametrize("case", range(max(16, N_CASES // 4)))
def test_sweep_pipeline(case):
    tables, cols, B, compact, thresholds = draw_pipeline(case)
    dt = [ccj.Table.from_host(kind, bk) for kind, bk in tables]
    ot = [O.Table(kind, bk) for kind, bk in tables]
    cf = max(max(1, int(t.max_dup)) for t in dt)
    want = oracle_pipeline(ot, cols, B, compact, cap_factor=cf, max_rounds=1 + max(int(t.max_rounds) for t in dt),
                           thresholds=thresholds)
    pl = ccj.Pipeline(dt, B, compact)
    if thresholds is not None:
        pl.set_thresholds(thresholds)
    pl.run([torch.from_numpy(c).cuda() for c in cols])
    joins = len(dt)
    got = pl.result_columns()
    got = got[:joins] + [got[joins + 2 * l + 1] for l in range(joins)]
    assert pl.res.n_out == len(want[0]), (pl.res.n_out, len(want[0]))
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)
