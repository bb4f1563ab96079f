"""Parity of the HIP probe path (through the C ABI) against the reference and the oracle.

  L3  every reference golden trace, replayed on device with the reference-order table
  L2  device-built (atomicCAS) LP tables vs the oracle: multiset of (global row, payload)
  L1+L2 at larger sizes via the exact membership oracle (size-independent)
  edge cases: empty input, ragged chunks, every chunk width, -1 keys, overflow flags
"""
import numpy as np
import pytest

from helpers import (assert_trace_equal, known_answers, load_trace, ref_keys, trace_inputs,
                     views_from_rounds)
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

KA = known_answers()
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


def to_dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to(DEV)


def host(o):
    torch.cuda.synchronize()
    return {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in o.items()}


def matches_of(out, chunk):
    """(global rows, payloads) of every match, in emission order."""
    n_chunks, cap = out["n_chunks"], out["cap"]
    cnt = out["count"].astype(np.int64)
    valid = np.arange(cap)[None, :] < cnt[:, None]
    sel = out["sel"].reshape(n_chunks, cap)[valid].astype(np.uint32).astype(np.uint64)
    pay = out["payload"].reshape(n_chunks, cap)[valid]
    rows = np.repeat(np.arange(n_chunks, dtype=np.uint64), cnt) * np.uint64(chunk) + sel
    return rows, pay


@pytest.mark.parametrize("name", sorted(KA["trace_cases"]))
def test_l3_reference_traces(name):
    entry = KA["trace_cases"][name]
    spec = entry["spec"]
    kind = ccj.LP if spec["kind"] == "lp" else ccj.CHAIN
    table = ccj.Table.reference(kind, spec["n_build"], spec["cf"], ccj.LAYOUT_REFERENCE)
    assert table.max_dup == min(spec["cf"], spec["n_build"])
    for view in entry["views"]:
        trace = load_trace(name, view)
        keys, sel, counts = trace_inputs(spec, trace)
        out = host(table.probe(to_dev(keys), spec["B"], sel=to_dev(sel.view(np.int32)),
                               counts=to_dev(counts.view(np.int32))))
        assert out["status"][0] == 0
        got = views_from_rounds(out["count"], out["sel"].view(np.uint32), out["payload"], out["rounds"],
                                out["round_counts"], out["cap"], out["max_rounds"], merged=(view == "merged"))
        assert_trace_equal(got, trace)


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
@pytest.mark.parametrize("chunk", [1, 63, 64, 65, 256, 1000, 2047, 2048])
def test_l3_every_chunk_width_vs_oracle(kind, chunk):
    bk = ref_keys(20000, 3)
    table = ccj.Table.from_host(kind, bk)
    otab = O.Table(kind, bk)
    keys = O.uniform_keys(11, 0, 50000, 30000)
    keys[::97] = -1  # the empty marker as a probe key never matches (slot == -1 ends the run)
    out = host(table.probe(to_dev(keys), chunk))
    want = otab.probe(keys, chunk, cap_factor=3, max_rounds=out["max_rounds"])
    assert out["status"][0] == 0
    for view_merged in (False, True):
        g = views_from_rounds(out["count"], out["sel"].view(np.uint32), out["payload"], out["rounds"],
                              out["round_counts"], out["cap"], out["max_rounds"], merged=view_merged)
        w = views_from_rounds(want["count"], want["sel"], want["payload"], want["rounds"], want["round_counts"],
                              want["cap"], want["max_rounds"], merged=view_merged)
        assert_trace_equal(g, w)


def test_empty_and_tiny_inputs():
    table = ccj.Table.reference(ccj.LP, 1000, 1)
    out = host(table.probe(torch.empty(0, dtype=torch.int64, device=DEV), 2048))
    assert out["n_chunks"] == 0
    out = host(table.probe(to_dev(np.array([5], np.int64)), 2048))
    assert out["count"][0] == 1 and out["sel"][0] == 0 and out["payload"][0] == 5
    # counts = 0 for a chunk: no active row, zero rounds
    keys = to_dev(np.arange(4096, dtype=np.int64))
    out = host(table.probe(keys, 2048, counts=to_dev(np.array([0, 2048], np.int32))))
    assert out["count"][0] == 0 and out["rounds"][0] == 0 and out["count"][1] == 0  # keys >= 1000 miss
    out = host(table.probe(keys, 2048, counts=to_dev(np.array([1000, 5], np.int32))))
    assert out["count"][0] == 1000 and out["count"][1] == 0


def test_overflow_and_bad_input_flags():
    table = ccj.Table.reference(ccj.LP, 4096, 4)
    keys = to_dev(O.uniform_keys(3, 0, 4096, 4096))
    out = host(table.probe(keys, 2048, cap=100))
    assert out["status"][0] & ccj.FLAG_CAP_OVERFLOW
    assert (out["count"] <= 100).all()
    o2 = table.alloc_outputs(4096, 2048)
    o2["max_rounds"] = 1
    out = host(table.probe(keys, 2048, out=o2))
    assert out["status"][0] & ccj.FLAG_ROUND_OVERFLOW
    sel = np.tile(np.arange(2048, dtype=np.int32), 2)
    sel[5] = 5000
    out = host(table.probe(keys, 2048, sel=to_dev(sel)))
    assert out["status"][0] & ccj.FLAG_BAD_INPUT


@pytest.mark.parametrize("cf", [1, 2, 5])
def test_l2_device_built_lp_vs_oracle(cf):
    n = 1 << 20
    d_keys = to_dev(ref_keys(n, cf))
    table = ccj.Table.on_device(ccj.LP, d_keys)
    otab = O.Table(O.LP, ref_keys(n, cf))
    probe = O.uniform_keys(99, 0, 4 << 20, 3 * n // 2)
    out = host(table.probe(to_dev(probe), 2048))
    assert out["status"][0] == 0
    rows, pay = matches_of(out, 2048)
    m, l2 = O.count_uniform(99, 0, 4 << 20, 3 * n // 2, n, cf)
    assert len(rows) == m
    assert O.l2_sum(rows, pay) == l2
    want = otab.probe(probe, 2048, cap_factor=cf, max_rounds=4096)
    assert table.max_rounds >= int(want["rounds"].max())
    assert int(out["rounds"].max()) == int(want["rounds"].max())  # rounds depend only on the occupied set


def test_device_lp_build_run_stats_match_host_layout():
    n = 1 << 18
    host_t = ccj.Table.reference(ccj.LP, n, 1, ccj.LAYOUT_REFERENCE)
    dev_t = ccj.Table.reference(ccj.LP, n, 1, ccj.LAYOUT_DEVICE)
    assert host_t.size == dev_t.size
    assert host_t.max_rounds == dev_t.max_rounds  # the occupied set is insertion-order independent


@pytest.mark.parametrize("n", [2, 3, 5, 9, 15])
@pytest.mark.parametrize("dups", [False, True])
def test_device_lp_build_tiny_table_wrapping_run(n, dups):
    """Tables of < 64 slots (n < 16 keys): a run that wraps round the table's end.  The device
    build's run statistics (lp_runs) must see the table end at slot size - 1, not at the step's bit
    63 — found by tests/test_sweep_gpu.py: 5 equal keys gave max_dup 4 and a short max_rounds."""
    size = 1
    while size < 4 * n:
        size <<= 1
    cand = np.arange(1, 1 << 16, dtype=np.int64)
    home = (_np_murmur(cand.astype(np.uint64)) & np.uint64(size - 1)).astype(np.int64)
    k0 = int(cand[home == size - 1][0])  # its run starts at the last slot and wraps
    keys = np.full(n, k0, np.int64) if dups else np.concatenate([[k0], cand[home == size - 1][1:n]])
    host_t = ccj.Table.from_host(ccj.LP, keys)
    dev_t = ccj.Table.on_device(ccj.LP, to_dev(keys))
    assert (dev_t.size, dev_t.max_rounds, dev_t.max_dup) == (host_t.size, host_t.max_rounds, host_t.max_dup)
    assert dev_t.max_rounds == n and dev_t.max_dup == (n if dups else 1)
    out = host(dev_t.probe(to_dev(keys), 64))
    assert out["status"][0] == 0 and int(out["count"][0]) == (n * n if dups else n)


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
def test_l1_l2_large_membership(kind):
    n, n_probe, rng = 1 << 22, 1 << 26, 3 << 21
    table = ccj.Table.reference(kind, n, 1, ccj.LAYOUT_DEVICE)
    keys = to_dev(O.uniform_keys(7, 0, n_probe, rng))
    out = table.probe(keys, 2048, rounds=False)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    cnt = out["count"].to(torch.int64)
    m, l2 = O.count_uniform(7, 0, n_probe, rng, n, 1)
    assert int(cnt.sum().item()) == m
    # L2 checksum computed on the device side of the test with torch integer ops
    rows, pay = matches_of(host(out), 2048)
    assert O.l2_sum(rows, pay) == l2


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("n_build,cf,n_probe,rng", [(1 << 20, 1, 1 << 22, 1 << 20), (1 << 22, 2, 1 << 23, 3 << 21),
                                                    (1 << 16, 1, 100000, 1 << 17), (1000, 1, 5000, 2000),
                                                    (1 << 24, 1, (1 << 24) + 77, 1 << 24)])
def test_partitioned_probe_l1_l2(n_build, cf, n_probe, rng, exact):
    table = ccj.Table.reference(ccj.LP, n_build, cf, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(n_probe, 31, rng)
    out = table.probe_partitioned(keys, 2048, exact=exact)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0 and not out.get("exact_retry")
    m, l2 = ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64))
    assert (m, l2) == O.count_uniform(31, 0, n_probe, rng, n_build, cf)
    if exact or out["row_map"].numel() == n_probe:
        # exact split (or one window): the row map is a permutation of the probe rows
        rm = out["row_map"][:n_probe].cpu().numpy().view(np.uint32)
        assert np.array_equal(np.sort(rm), np.arange(n_probe, dtype=np.uint32))


@pytest.mark.parametrize("n_build,n_probe,rng", [(1 << 20, 1 << 22, 1 << 20), (1 << 20, 1 << 22, 3 << 19),
                                                (5000, 70000, 20000), (100, 5000, 100), (1 << 16, 1000, 1 << 18)])
@pytest.mark.parametrize("exact", [False, True])
def test_partitioned_probe_rows_mode(n_build, n_probe, rng, exact):
    """CCJ_PART_ROWS (distinct keys, cap == chunk): the split writes every position's key into
    out_payload and its original row into out_sel; the walk compacts only the chunks with misses.
    rng == n_build: every row matches (no chunk is touched by the walk's emit); larger ranges mix
    full chunks and compacted ones.  Exact L1 + L2 with sel read as global rows, and every output
    pair (row, payload) is the row's own key."""
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(n_probe, 37, rng)
    out = table.probe_partitioned(keys, 2048, exact=exact, rows=True)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0 and out["row_map"] is None
    assert ccj.result_checksum(out, 0) == O.count_uniform(37, 0, n_probe, rng, n_build, 1)
    cnt = out["count"][:out["n_chunks"]].cpu().numpy().view(np.uint32).astype(np.int64)
    cap = out["cap"]
    idx = (np.arange(len(cnt))[:, None] * cap + np.arange(2048)[None, :])[np.arange(2048)[None, :] < cnt[:, None]]
    sel = out["sel"].cpu().numpy().view(np.uint32)[idx].astype(np.int64)
    pay = out["payload"].cpu().numpy()[idx]
    k = keys.cpu().numpy()
    assert np.array_equal(pay, k[sel])  # payload = the matched row's key
    assert len(np.unique(sel)) == len(sel)  # distinct keys: each row at most once


def test_partitioned_probe_payload_aliasing_off_matches_on():
    """cap == chunk without CCJ_PART_ROWS: the keys go straight to out_payload; the outputs (per chunk
    counts, sel, payload) are the same multiset as with the workspace key column (cap > chunk)."""
    table = ccj.Table.reference(ccj.LP, 1 << 16, 1, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(1 << 20, 41, 3 << 15)
    a = table.probe_partitioned(keys, 2048)
    b = table.probe_partitioned(keys, 2048, cap=4096)
    torch.cuda.synchronize()
    assert a["cap"] == 2048 and b["cap"] == 4096
    want = O.count_uniform(41, 0, 1 << 20, 3 << 15, 1 << 16, 1)
    assert ccj.result_checksum(a, 2048, row_map=a["row_map"].to(torch.int64)) == want
    assert ccj.result_checksum(b, 2048, row_map=b["row_map"].to(torch.int64)) == want


@pytest.mark.parametrize("n_build,cf,n_probe,rng", [(1 << 20, 1, 1 << 22, 1 << 20), (1 << 16, 3, 300000, 1 << 17),
                                                    (5000, 1, 70000, 20000), (4096, 64, 100000, 8192),
                                                    (3, 1, 5000, 6), (1 << 19, 2, 1 << 21, 3 << 19)])
@pytest.mark.parametrize("positions", [False, True])
def test_partitioned_probe_walks(n_build, cf, n_probe, rng, positions):
    """The partitioned walks give the exact L1 + L2 answer: probe_walk (match counts, wave-ordered
    emit) and, with match positions requested, probe_win (C5); duplicates (cf 3, cf 64: runs far
    longer than 32 slots), misses, a tiny table (identity layout) and a table of exactly one
    window included."""
    table = ccj.Table.reference(ccj.LP, n_build, cf, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(n_probe, 17, rng)
    kw = dict(pos=True) if positions and table.size >= 16 else {}
    out = table.probe_partitioned(keys, 2048, **kw)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    m, l2 = ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64))
    assert (m, l2) == O.count_uniform(17, 0, n_probe, rng, n_build, cf)
    if kw:  # every recorded position holds the matched key
        h = host(out)
        tab = table_slots(table)
        valid = np.arange(h["cap"])[None, :] < h["count"].astype(np.int64)[:, None]
        pos = h["pos"].reshape(-1, h["cap"])[valid].view(np.uint32)
        assert np.array_equal(tab[pos], h["payload"].reshape(-1, h["cap"])[valid])


def table_slots(table):
    """The device table's slot array on the host (LP)."""
    import ctypes as C
    out = np.empty(max(table.size, 4), np.int64)
    from ccj import _d2h_i64
    return _d2h_i64(table.d_table, len(out))


@pytest.mark.parametrize("distinct", [1, 7, 3000])
def test_partitioned_probe_skew_falls_back_to_exact(distinct):
    """Heavy skew overflows the one-pass split's fixed segments and then its overflow area (n/16
    rows): the ABI raises FLAG_PART_OVERFLOW (rows dropped) and the wrapper re-runs with the exact
    split.  A handful of distinct keys cannot fit; 3000 keys over 3·2^20 probes may."""
    n_build, n_probe = 1 << 20, (1 << 24) if distinct <= 7 else 3 << 20
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    g = np.random.default_rng(distinct)
    vals = g.integers(0, 2 * n_build, size=distinct)
    keys_h = vals[g.integers(0, distinct, size=n_probe)].astype(np.int64)
    keys = torch.from_numpy(keys_h).cuda()
    raw = table.probe_partitioned(keys, 2048, retry=False)
    torch.cuda.synchronize()
    overflow = bool(int(raw["status"].item()) & ccj.FLAG_PART_OVERFLOW)
    out = table.probe_partitioned(keys, 2048)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    assert bool(out.get("exact_retry")) == overflow
    if distinct <= 7:
        assert overflow  # a handful of keys cannot spread over the partitions' segments and the overflow area
    # expected answer by membership (reference generator: every key < n_build matches once)
    hit = keys_h < n_build
    rows = np.nonzero(hit)[0].astype(np.uint64)
    want = (len(rows), O.l2_sum(rows, keys_h[hit]))
    assert ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64)) == want


@pytest.mark.parametrize("rows", [False, True])
def test_partitioned_probe_skew_few_tiles_stays_one_pass(rows):
    """Fewer rows than 8 split tiles: only some tile groups (XCDs) receive tiles, so each group's
    overflow sub-area is sized from the rows one group can get, not 1/8 of the area.
    40 % of the rows are one hot key: its run outgrows the partition's segment in every tile and
    fits the group's sub-area — no exact-split fallback, exact L1 + L2."""
    n_build, n_probe = 1 << 20, 30000
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    g = np.random.default_rng(77)
    keys_h = g.integers(0, 2 * n_build, size=n_probe).astype(np.int64)
    keys_h[g.random(n_probe) < 0.4] = 4242
    keys = torch.from_numpy(keys_h).cuda()
    out = table.probe_partitioned(keys, 2048, retry=False, rows=rows)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    hit = keys_h < n_build
    r = np.nonzero(hit)[0].astype(np.uint64)
    want = (len(r), O.l2_sum(r, keys_h[hit]))
    got = ccj.result_checksum(out, 0) if rows else \
        ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64))
    assert got == want


def test_partitioned_probe_same_rows_as_chunk_probe():
    n_build, n_probe = 1 << 20, 1 << 21
    table = ccj.Table.reference(ccj.LP, n_build, 3, ccj.LAYOUT_REFERENCE)
    keys = ccj.gen_uniform_keys(n_probe, 5, n_build)
    a = host(table.probe(keys, 2048))
    b = host(table.probe_partitioned(keys, 2048))
    ra, pa = matches_of(a, 2048)
    rb_local, pb = matches_of(b, 2048)
    rb = b["row_map"].view(np.uint32)[rb_local.astype(np.int64)].astype(np.uint64)
    oa = np.lexsort((pa, ra))
    ob = np.lexsort((pb, rb))
    assert np.array_equal(ra[oa], rb[ob]) and np.array_equal(pa[oa], pb[ob])


@pytest.mark.parametrize("kind", [0, 1])
def test_device_build_reports_exact_max_dup(kind):
    """Probe outputs are sized by max_dup (cap = chunk * max_dup): a device-built table reports the
    exact largest multiplicity of one key, not a bound."""
    rng = np.random.default_rng(3)
    base = rng.integers(0, 1 << 40, size=5000)
    reps = rng.integers(1, 4, size=5000)
    reps[1234] = 9
    keys = np.repeat(base, reps)
    rng.shuffle(keys)
    t = ccj.Table.on_device(kind, torch.from_numpy(keys).cuda())
    assert t.max_dup == 9
    out = t.probe(torch.from_numpy(base).cuda(), 2048)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    assert int(out["count"].sum().item()) == int(reps.sum())


@pytest.mark.parametrize("exact", [False, True])
@pytest.mark.parametrize("n_build,cf,n_probe,rng", [(1 << 20, 1, 1 << 22, 1 << 21), (1 << 18, 3, 1 << 21, 1 << 19),
                                                    (3000, 2, 40000, 9000), (1 << 22, 3, 3 << 21, 3 << 22),
                                                    (1 << 21, 1, (1 << 22) + 4097, 10 << 21),
                                                    (5 << 20, 2, 1 << 23, 5 << 20), (1 << 20, 2, 1 << 22, 1 << 20)])
def test_partitioned_chaining_probe_l1_l2(n_build, cf, n_probe, rng, exact):
    """Bucket-range-partitioned chaining probe — exact L1 + L2 against the membership answer,
    duplicates and misses included.  Tables of >= 8 partitions take probe_chain_filt (the
    partition's 2-bit bucket filter in LDS, quarter-chunk work units, the overflow area by
    probe_chain_win); smaller ones and the exact split probe_chain_win alone (bucket record, then
    2-key windows of the CSR chain).  Shapes: 8 / 32 / 64 partitions, 90 % misses, ragged last
    chunk, cf 2 / 3, and every row a hit (all 256 rows of a filter-walk unit in its chain queue:
    four queue passes per unit)."""
    table = ccj.Table.reference(ccj.CHAIN, n_build, cf, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(n_probe, 23, rng)
    out = table.probe_partitioned(keys, 2048, exact=exact)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    m, l2 = ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64))
    assert (m, l2) == O.count_uniform(23, 0, n_probe, rng, n_build, cf)


@pytest.mark.parametrize("n_build,n_probe", [(1 << 20, 1 << 22), (1 << 23, 1 << 24)])
def test_partitioned_chaining_c3_skew(n_build, n_probe):
    """C3's Zipf-skewed hits overflow the fixed split (hot keys pile into one partition's segments
    and then the shared overflow area, which probe_chain_win walks beside the filter walk); the
    exact split and the chain walks still give the exact answer."""
    table = ccj.Table.reference(ccj.CHAIN, n_build, 1, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_c3_keys(n_probe, 42, n_build, 1)
    out = table.probe_partitioned(keys, 2048)  # retries with the exact split on overflow
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    if n_build >= 1 << 23:  # 64 partitions: the hot keys spill into the overflow area, which holds them
        assert not out.get("exact_retry")
    m, l2 = ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64))
    assert (m, l2) == O.count_c3(42, 0, n_probe, n_build, 1)


@pytest.mark.parametrize("n_build", [1 << 20, 5000])
def test_partitioned_probe_chunk_counts(n_build):
    """Segmented input (the multi-GPU receive buffers): only the first counts[c] rows of chunk c
    are live; the dead rows hold keys that WOULD match and must not be probed."""
    chunk, n_chunks = 2048, 700
    rng = np.random.default_rng(5)
    keys_h = rng.integers(0, n_build, size=n_chunks * chunk).astype(np.int64)  # every key a hit
    counts_h = rng.integers(0, chunk + 1, size=n_chunks).astype(np.uint32)
    counts_h[::7] = chunk
    counts_h[3::11] = 0
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    counts = torch.from_numpy(counts_h.view(np.int32)).cuda()
    out = table.probe_partitioned(torch.from_numpy(keys_h).cuda(), chunk, counts=counts)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    pos = np.arange(n_chunks * chunk)
    live = (pos % chunk) < counts_h[pos // chunk]
    want = (int(live.sum()), O.l2_sum(pos[live].astype(np.uint64), keys_h[live]))
    assert ccj.result_checksum(out, chunk, row_map=out["row_map"].to(torch.int64)) == want


def test_c2_table_size_reference_vector():
    """The reference's own answer at C2's table size (SURVEY §4 survey_lp_2048_64M_64M: a 2^26-key
    LP table = 2^28 slots = 2 GiB, 2^26 mt19937_64(42) probe keys % 2^26, B = 2048).
    Chunk path on the reference-order table: matches, L2, the ordered L3 fold and the SURVEY
    checksum equal the reference's (L3).  Partitioned path (bench.py's headline) on a device-built
    table: matches and L2 equal it (L1 + L2)."""
    entry = KA["sum_cases"]["survey_lp_2048_64M_64M"]
    spec, want = entry["spec"], entry["variants"]["next"]
    n, B = spec["n_build"], spec["B"]
    keys = to_dev(O.mt64_keys(spec["seed"], spec["n_probe"], spec["range"]))
    table = ccj.Table.reference(ccj.LP, n, spec["cf"], ccj.LAYOUT_REFERENCE)
    assert table.size == 1 << 28
    out = host(table.probe(keys, B, rounds=False))
    assert out["status"][0] == 0
    got = O.result_sums(out["count"], out["sel"], out["payload"], out["cap"], B)
    assert got == (want["matches"], want["l2"], want["l3"], want["survey_chk"])
    table.free()
    del out
    table = ccj.Table.reference(ccj.LP, n, spec["cf"], ccj.LAYOUT_DEVICE)
    pout = table.probe_partitioned(keys, B)
    torch.cuda.synchronize()
    assert int(pout["status"].item()) == 0
    assert ccj.result_checksum(pout, B, row_map=pout["row_map"].to(torch.int64)) == (want["matches"], want["l2"])
    table.free()


@pytest.mark.parametrize("layout", [ccj.LAYOUT_REFERENCE, ccj.LAYOUT_DEVICE])
@pytest.mark.parametrize("n_build,cf,n_probe,rng,chunk,ragged", [
    (1 << 20, 1, 1 << 22, 1 << 20, 2048, False),
    (1 << 20, 3, 3000000, 3 << 19, 2048, True),
    (1 << 20, 1, 1 << 21, 5 << 20, 256, False),       # 80 % misses, the reference's default chunk
    (1 << 20, 1, 999999, 1 << 20, 1000, True),        # ragged chunks of an odd width
    (1 << 20, 40, 1 << 20, 1 << 20, 2048, False),     # runs longer than 26 rounds: re-walked chunks
])
def test_ordered_probe_equals_chunk_probe(layout, n_build, cf, n_probe, rng, chunk, ragged):
    """ccj_probe_ordered (split -> round words -> back to row order -> emit) gives exactly
    ccj_probe's outputs: per-chunk counts, rounds, every Next's count and the ordered
    (sel, payload) stream (L3)."""
    table = ccj.Table.reference(ccj.LP, n_build, cf, layout)
    assert table.size >= 1 << 22
    keys = ccj.gen_uniform_keys(n_probe, 23, rng)
    counts = None
    if ragged:
        n_chunks = -(-n_probe // chunk)
        g = np.random.default_rng(cf)
        c = g.integers(0, chunk + 1, size=n_chunks).astype(np.int32)
        c[::5] = chunk
        c[-1] = min(c[-1], n_probe - (n_chunks - 1) * chunk)
        counts = to_dev(c)
    want = host(table.probe(keys, chunk, counts=counts))
    got = host(table.probe_ordered(keys, chunk, counts=counts))
    assert got["status"][0] == 0 and want["status"][0] == 0
    assert np.array_equal(got["count"], want["count"])
    assert np.array_equal(got["rounds"], want["rounds"])
    assert np.array_equal(got["round_counts"], want["round_counts"])
    cap = want["cap"]
    valid = np.arange(cap)[None, :] < want["count"].astype(np.int64)[:, None]
    assert np.array_equal(got["sel"].reshape(-1, cap)[valid], want["sel"].reshape(-1, cap)[valid])
    assert np.array_equal(got["payload"].reshape(-1, cap)[valid], want["payload"].reshape(-1, cap)[valid])


@pytest.mark.parametrize("n_build,cf,n_probe,chunk,ragged,c3", [
    (1 << 21, 1, 1 << 22, 2048, False, True),    # C3's stream: 10 % Zipf hits, 90 % misses
    (1 << 21, 3, 3000000, 2048, True, True),     # duplicate keys (32-bit round words), ragged chunks
    (1 << 21, 1, 999999, 1000, True, False),     # uniform hits, odd chunk width, ragged
    (1 << 21, 1, 1 << 21, 256, False, False),    # the reference's default chunk
    (1 << 21, 40, 1 << 20, 2048, False, False),  # chains longer than 26 nodes: re-walked chunks
])
def test_ordered_probe_chaining_equals_chunk_probe(n_build, cf, n_probe, chunk, ragged, c3):
    """ccj_probe_ordered on a chaining table (bucket split -> round words from the chain walk ->
    back to row order -> emit) gives exactly probe_chunks<CHAIN>'s outputs: per-chunk counts,
    rounds, every Next's count and the ordered (sel, payload) stream (L3)."""
    table = ccj.Table.reference(ccj.CHAIN, n_build, cf, ccj.LAYOUT_REFERENCE)
    assert table.size >= 1 << 22
    keys = (ccj.gen_c3_keys(n_probe, 29, n_build, cf) if c3 else
            ccj.gen_uniform_keys(n_probe, 31, n_build * 2 // cf + 1))
    counts = None
    if ragged:
        n_chunks = -(-n_probe // chunk)
        g = np.random.default_rng(cf + 7)
        c = g.integers(0, chunk + 1, size=n_chunks).astype(np.int32)
        c[::5] = chunk
        c[-1] = min(c[-1], n_probe - (n_chunks - 1) * chunk)
        counts = to_dev(c)
    want = host(table.probe(keys, chunk, counts=counts))
    got = host(table.probe_ordered(keys, chunk, counts=counts))
    assert got["status"][0] == 0 and want["status"][0] == 0 and not got.get("exact_retry")
    assert want["count"].sum() > 0
    assert np.array_equal(got["count"], want["count"])
    assert np.array_equal(got["rounds"], want["rounds"])
    assert np.array_equal(got["round_counts"], want["round_counts"])
    cap = want["cap"]
    valid = np.arange(cap)[None, :] < want["count"].astype(np.int64)[:, None]
    assert np.array_equal(got["sel"].reshape(-1, cap)[valid], want["sel"].reshape(-1, cap)[valid])
    assert np.array_equal(got["payload"].reshape(-1, cap)[valid], want["payload"].reshape(-1, cap)[valid])


@pytest.mark.parametrize("kind", ["lp", "chain"])
@pytest.mark.parametrize("chunk,n_probe", [(1, 500), (4, 400), (7, 20), (64, 300)])
def test_ordered_probe_small_inputs_equal_chunk_probe(kind, chunk, n_probe):
    """Tiny chunks and few rows: the overflow area is then under 128 positions, so the ordered
    route's split is the non-pipelined slot_split_fixed, which must leave each row's tile index
    at its IMAGE position as the pipelined split does (it wrote it at the segment
    destination, and the unsplit read stale workspace). L3 against ccj_probe."""
    if kind == "lp":
        table = ccj.Table.reference(ccj.LP, 1 << 20, 1, ccj.LAYOUT_REFERENCE)
        keys = ccj.gen_uniform_keys(n_probe, 41 + chunk, 3 << 19)
    else:
        table = ccj.Table.reference(ccj.CHAIN, 1 << 21, 3, ccj.LAYOUT_REFERENCE)
        keys = ccj.gen_uniform_keys(n_probe, 43 + chunk, (1 << 21) // 3)
    assert table.size >= 1 << 22
    want = host(table.probe(keys, chunk))
    got = host(table.probe_ordered(keys, chunk))
    assert got["status"][0] == 0 and want["status"][0] == 0 and not got.get("exact_retry")
    assert want["count"].sum() > 0
    assert np.array_equal(got["count"], want["count"])
    assert np.array_equal(got["rounds"], want["rounds"])
    assert np.array_equal(got["round_counts"], want["round_counts"])
    cap = want["cap"]
    valid = np.arange(cap)[None, :] < want["count"].astype(np.int64)[:, None]
    assert np.array_equal(got["sel"].reshape(-1, cap)[valid], want["sel"].reshape(-1, cap)[valid])
    assert np.array_equal(got["payload"].reshape(-1, cap)[valid], want["payload"].reshape(-1, cap)[valid])
    table.free()


def test_ordered_probe_c2_table_reference_vector():
    """ccj_probe_ordered on the reference-order 2^26-key table against the reference's own vector
    (SURVEY §4 survey_lp_2048_64M_64M): matches, L2, the ordered L3 fold, the SURVEY checksum."""
    entry = KA["sum_cases"]["survey_lp_2048_64M_64M"]
    spec, want = entry["spec"], entry["variants"]["next"]
    keys = to_dev(O.mt64_keys(spec["seed"], spec["n_probe"], spec["range"]))
    table = ccj.Table.reference(ccj.LP, spec["n_build"], spec["cf"], ccj.LAYOUT_REFERENCE)
    out = host(table.probe_ordered(keys, spec["B"], rounds=False))
    assert out["status"][0] == 0 and not out.get("exact_retry")
    assert O.result_sums(out["count"], out["sel"], out["payload"], out["cap"], spec["B"]) == \
        (want["matches"], want["l2"], want["l3"], want["survey_chk"])
    table.free()


def test_ordered_probe_skew_retries_chunk_path():
    """Extreme skew overflows the split's overflow area: the wrapper re-runs ccj_probe."""
    n_build, n_probe = 1 << 20, 3 << 20
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_REFERENCE)
    keys = torch.full((n_probe,), 12345, dtype=torch.int64, device=DEV)
    want = host(table.probe(keys, 2048))
    got = host(table.probe_ordered(keys, 2048))
    assert got["status"][0] == 0 and got.get("exact_retry")
    assert np.array_equal(got["count"], want["count"]) and np.array_equal(got["sel"], want["sel"])


def _np_murmur(x):
    """hash_functions.h:8-16 on a uint64 array (wrapping multiplies)."""
    x = x.astype(np.uint64)
    c = np.uint64(0xd6e8feb86659fd93)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(32)
        x *= c
        x ^= x >> np.uint64(32)
        x *= c
        x ^= x >> np.uint64(32)
    return x


@pytest.mark.parametrize("mode", ["rows", "positions", "plain", "payload"])
def test_partitioned_walk_long_runs_across_windows(mode):
    """probe_walk2 (distinct keys: a row ends at its match, phase B for rows whose run goes on) on
    runs hundreds of keys long that cross a 2^19-slot window's end and wrap around the table's:
    a host-built table of 2^18 keys in 2^20 slots with 400-key clusters hashed just below each
    window's end.  Probes: every build key, repeats, misses (which walk whole clusters) and the
    cluster keys again.  L1 + L2 exact in rows mode, with positions (every position holds its key),
    in plain mode (row map) and with payload columns (CCJ_PART_ROWS + walk2<POS> + gather)."""
    g = np.random.default_rng(11)
    size = 1 << 20
    cand = np.unique(g.integers(1, 1 << 40, size=1 << 24, dtype=np.int64))
    g.shuffle(cand)
    home = (_np_murmur(cand.astype(np.uint64)) & np.uint64(size - 1)).astype(np.int64)
    edge0 = cand[(home >= (1 << 19) - 96) & (home < (1 << 19))][:400]
    edge1 = cand[(home >= size - 96)][:400]
    assert len(edge0) == 400 and len(edge1) == 400
    rest = np.setdiff1d(cand[:600000], np.concatenate([edge0, edge1]))
    n_build = 1 << 18
    build = np.concatenate([edge0, edge1, rest[:n_build - 800]])
    g.shuffle(build)
    table = ccj.Table.from_host(ccj.LP, build)
    assert table.size == size and int(table.max_dup) == 1
    pk = np.concatenate([build, build[:1000], rest[n_build:n_build + 50000], edge0, edge1, edge1])
    g.shuffle(pk)
    keys = torch.from_numpy(pk).cuda()
    hit = np.isin(pk, build)
    r = np.nonzero(hit)[0].astype(np.uint64)
    want = (len(r), O.l2_sum(r, pk[hit]))
    if mode == "payload":
        pay = (build.astype(np.int64)[:, None] * 3 + np.arange(8, dtype=np.int64)[None, :]).reshape(-1)
        table.set_payload(torch.from_numpy(pay).cuda(), 8)
        out = table.probe_partitioned(keys, 2048, rows=True, pos=True, payload_cols=8)
    else:
        out = table.probe_partitioned(keys, 2048, rows=mode != "plain", pos=mode == "positions")
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    if mode == "plain":
        assert ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64)) == want
    else:
        assert ccj.result_checksum(out, 0) == want
    if mode in ("positions", "payload"):
        nc, cap = out["n_chunks"], out["cap"]
        cnt = out["count"][:nc].to(torch.int64).cpu().numpy()
        valid = (np.arange(cap)[None, :] < cnt[:, None]).reshape(-1)
        pos = out["pos"].cpu().numpy()[:nc * cap].view(np.uint32)[valid]
        key = out["payload"].cpu().numpy()[:nc * cap][valid]
        slots = np.full(size, -1, np.int64)
        # the table's slot array, host-built in the reference's order
        for k in build:
            s = int(_np_murmur(np.array([k], np.uint64))[0] & np.uint64(size - 1))
            while slots[s] != -1:
                s = (s + 1) & (size - 1)
            slots[s] = k
        assert np.array_equal(slots[pos], key)  # every recorded position holds its row's key
        if mode == "payload":
            for c in (0, 7):
                col = out["payload_cols"][c].cpu().numpy()[:nc * cap][valid]
                assert np.array_equal(col, key * 3 + c)
    table.free()


@pytest.mark.parametrize("chunk", [1, 7, 64, 100, 511, 512, 1000, 1024, 1536, 2047])
def test_partitioned_distinct_keys_every_chunk_width(chunk):
    """probe_walk2 (distinct keys) with chunks that leave waves partly or wholly empty (a wave owns
    512 rows of a chunk): rows mode, plain mode with the row map, and positions, each with misses
    (1/5 of the probes) and a ragged last chunk.  Exact L1 + L2; rows mode: every (row, payload)
    pair is the row's own key."""
    n_build, n_probe, rng = 1 << 18, 300007, (1 << 18) + (1 << 16)
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    assert int(table.max_dup) == 1
    keys = ccj.gen_uniform_keys(n_probe, 71, rng)
    want = O.count_uniform(71, 0, n_probe, rng, n_build, 1)
    out = table.probe_partitioned(keys, chunk, rows=True)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    assert ccj.result_checksum(out, 0) == want
    cnt = out["count"][:out["n_chunks"]].cpu().numpy().view(np.uint32).astype(np.int64)
    cap = out["cap"]
    idx = (np.arange(len(cnt))[:, None] * cap + np.arange(cap)[None, :])[np.arange(cap)[None, :] < cnt[:, None]]
    sel = out["sel"].cpu().numpy().view(np.uint32)[idx].astype(np.int64)
    assert np.array_equal(out["payload"].cpu().numpy()[idx], keys.cpu().numpy()[sel])
    out = table.probe_partitioned(keys, chunk, pos=True)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    assert ccj.result_checksum(out, chunk, row_map=out["row_map"].to(torch.int64)) == want
    table.free()


def test_partitioned_distinct_keys_rounds_walk_whole_runs():
    """With out_rounds asked for, the partitioned walk of a distinct-key table still walks every row
    to the end of its run (no early end at the match): each chunk's rounds equal the longest run,
    from the row's home slot to the first empty one, over the chunk's rows (the reference's Next
    calls for the chunk).  Every probe hits, so a chunk's count is its number of live rows."""
    n_build, n_probe = 1 << 18, 1 << 20
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    assert int(table.max_dup) == 1
    keys = ccj.gen_uniform_keys(n_probe, 91, n_build)
    out = table.probe_partitioned(keys, 2048, rounds=True)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    slots = table_slots(table)[:table.size]
    occ = slots != -1
    # run length from every slot: occupied slots from it up to the first empty one (with wrap)
    size = len(slots)
    runlen = np.zeros(size, np.int64)
    first_empty = int(np.nonzero(~occ)[0][0])
    run = 0
    for s in range(first_empty - 1 + size, first_empty - 1, -1):  # backwards, starting at an empty slot
        i = s % size
        run = run + 1 if occ[i] else 0
        runlen[i] = run
    k = keys.cpu().numpy()
    home = (_np_murmur(k.astype(np.uint64)) & np.uint64(size - 1)).astype(np.int64)
    nc = out["n_chunks"]
    cnt = out["count"][:nc].cpu().numpy().view(np.uint32).astype(np.int64)
    rounds = out["rounds"][:nc].cpu().numpy().view(np.uint32).astype(np.int64)
    rm = out["row_map"].cpu().numpy().view(np.uint32).astype(np.int64)
    assert cnt.sum() == n_probe
    for c in np.nonzero(cnt)[0]:
        rows = rm[c * 2048:c * 2048 + cnt[c]]
        assert rounds[c] == runlen[home[rows]].max(), c
    table.free()
