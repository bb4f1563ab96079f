"""The chaining hash table built on the device (csrc/ccj_build.hip) against the host
build in the reference's insertion order (chaining_ht.cpp:4-36: push_back per bucket).

  byte-identical: CSR offsets, chain keys, row map, 16- and 8-byte bucket records, longest chain
                  and max_dup of ccj_table_build_on_device(CHAIN) == ccj_table_build_from_host(CHAIN)
  L3:             every chain golden trace replayed on a table built by ccj_table_build_on_device
  no 8-byte records: a chain of >= 255 keys (the 16-byte record path of the ordered and partitioned
                  chain walks) — ordered == probe_chunks<CHAIN>, partitioned L1 + L2
"""
import numpy as np
import pytest

from helpers import assert_trace_equal, known_answers, load_trace, ref_keys, trace_inputs, views_from_rounds
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


def _keys(case):
    g = np.random.default_rng(7)
    if case == "empty":
        return np.zeros(0, np.int64)
    if case == "one":
        return np.array([42], np.int64)
    if case == "three":
        return np.array([5, -1, 5], np.int64)
    if case == "ref_cf1":
        return ref_keys(100000, 1)
    if case == "ref_cf7":
        return ref_keys(300001, 7)
    if case == "random_dups":  # shuffled multiplicities 1..9, 64-bit keys, -1 included
        base = g.integers(-1, 1 << 62, size=40000)
        reps = g.integers(1, 4, size=40000)
        reps[77] = 9
        k = np.repeat(base, reps)
        g.shuffle(k)
        return k.astype(np.int64)
    if case == "long_chain":  # one chain of 300 equal keys: no 8-byte records
        k = np.concatenate([ref_keys(5000, 1), np.full(300, 1234, np.int64)])
        g.shuffle(k)
        return k
    if case == "all_equal":  # one chain of every key: the radix sort skips every pass, max_dup = n
        return np.full(70000, -5, np.int64)
    if case == "wide_dups":  # keys over all 64 bits (every byte of the max_dup sort varies), dups 1..6
        base = g.integers(-(1 << 63), (1 << 63) - 1, size=150000, dtype=np.int64)
        k = np.repeat(base, g.integers(1, 6, size=150000))
        k = np.concatenate([k, np.full(6, base[3], np.int64)])
        g.shuffle(k)
        return k
    if case == "c3_size":  # 2^22 reference keys (C3 / C4 per-GPU shape, scaled)
        return ref_keys(1 << 22, 1)
    raise ValueError(case)


def _assert_same(host_t, dev_t):
    assert (dev_t.size, dev_t.n_keys, dev_t.max_rounds, dev_t.max_dup) == \
        (host_t.size, host_t.n_keys, host_t.max_rounds, host_t.max_dup)
    a, b = host_t.arrays(), dev_t.arrays()
    for k in ("table", "row", "off", "bucket16"):
        assert a[k].shape == b[k].shape, k
        assert np.array_equal(a[k], b[k]), (k, int(np.flatnonzero(a[k] != b[k])[0]))
    for k in ("bucket8", "filter"):
        assert (a[k] is None) == (b[k] is None), k
        if a[k] is not None:
            assert np.array_equal(a[k], b[k]), k
    if a["filter"] is not None:  # the filter model: 0 empty, 1 / 2 one key (hash bit 40), 3 longer
        ln = np.diff(a["off"].astype(np.int64))
        bit = (_np_murmur(a["table"][a["off"][:-1].astype(np.int64) % len(a["table"])]) >> np.uint64(40)) & np.uint64(1)
        code = np.where(ln == 0, 0, np.where(ln == 1, 1 + bit.astype(np.int64), 3)).astype(np.uint64)
        words = (code.reshape(-1, 16) << (2 * np.arange(16, dtype=np.uint64))[None, :]).sum(axis=1)
        assert np.array_equal(a["filter"].astype(np.uint64), words)
    return a


@pytest.mark.parametrize("case", ["empty", "one", "three", "ref_cf1", "ref_cf7", "random_dups", "long_chain",
                                  "all_equal", "wide_dups", "c3_size"])
def test_device_chain_build_byte_identical_to_host(case):
    keys = _keys(case)
    host_t = ccj.Table.from_host(ccj.CHAIN, keys)
    dev_t = ccj.Table.on_device(ccj.CHAIN, torch.from_numpy(keys).to(DEV))
    assert dev_t.layout == ccj.LAYOUT_DEVICE and host_t.layout == ccj.LAYOUT_REFERENCE
    a = _assert_same(host_t, dev_t)
    if len(keys):  # the CSR is the reference's std::list order: chain b = keys of bucket b in input order
        h = _np_murmur(keys) & np.uint64(host_t.size - 1)
        order = np.argsort(h, kind="stable")
        assert np.array_equal(a["row"][:len(keys)], order.astype(np.uint32))
        assert np.array_equal(a["table"][:len(keys)], keys[order])
    if case == "long_chain":
        assert a["bucket8"] is None and host_t.max_dup == 301 and host_t.max_rounds >= 301
    if case == "random_dups":
        assert host_t.max_dup == 9
    if case == "all_equal":
        assert dev_t.max_dup == 70000 and dev_t.max_rounds == 70000
    if case == "wide_dups":
        assert dev_t.max_dup == int(np.unique(keys, return_counts=True)[1].max())


@pytest.mark.parametrize("n,cf", [(1000, 1), (1 << 20, 1), (1 << 20, 3), (999999, 40)])
def test_reference_chain_build_is_the_device_build(n, cf):
    """ccj_table_build_reference(CHAIN, ...) — both layouts — runs the device build (generator on
    the device, max_dup from the generator) and equals the host build of the same keys."""
    host_t = ccj.Table.from_host(ccj.CHAIN, ref_keys(n, cf))
    for layout in (ccj.LAYOUT_DEVICE, ccj.LAYOUT_REFERENCE):
        dev_t = ccj.Table.reference(ccj.CHAIN, n, cf, layout)
        assert dev_t.layout == layout
        _assert_same(host_t, dev_t)


@pytest.mark.parametrize("name", sorted(k for k in KA["trace_cases"] if KA["trace_cases"][k]["spec"]["kind"] == "chain"))
def test_l3_chain_traces_on_device_built_table(name):
    """Every chaining golden trace (recorded from the reference) replayed on a table whose CSR was
    built by ccj_table_build_on_device from the reference generator's keys (L3)."""
    entry = KA["trace_cases"][name]
    spec = entry["spec"]
    table = ccj.Table.on_device(ccj.CHAIN, torch.from_numpy(ref_keys(spec["n_build"], spec["cf"])).to(DEV))
    assert table.max_dup == min(spec["cf"], spec["n_build"])
    for view in entry["views"]:
        trace = load_trace(name, view)
        keys, sel, counts = trace_inputs(spec, trace)
        out = table.probe(torch.from_numpy(keys).to(DEV), spec["B"], sel=torch.from_numpy(sel.view(np.int32)).to(DEV),
                          counts=torch.from_numpy(counts.view(np.int32)).to(DEV))
        torch.cuda.synchronize()
        h = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
        assert h["status"][0] == 0
        got = views_from_rounds(h["count"], h["sel"].view(np.uint32), h["payload"], h["rounds"], h["round_counts"],
                                h["cap"], h["max_rounds"], merged=(view == "merged"))
        assert_trace_equal(got, trace)


def test_chain_without_8_byte_records_ordered_and_partitioned():
    """A table with one chain of 300 equal keys has no 8-byte bucket records, so the chain walks take
    round 0 from the 16-byte records (ccj_kernels.hip chain_words / probe_chain_win fallback).
    Ordered probe == probe_chunks<CHAIN> output for output (L3); partitioned probe L1 + L2."""
    n = 1 << 21
    hot = 1 << 40
    build = np.concatenate([ref_keys(n, 1), np.full(299, hot, np.int64)])
    np.random.default_rng(3).shuffle(build)
    table = ccj.Table.on_device(ccj.CHAIN, torch.from_numpy(build).to(DEV))
    assert table.size >= 1 << 22 and table.arrays()["bucket8"] is None and table.max_dup == 299
    n_probe = 1 << 16  # cap = chunk * 299 per chunk: keep the chunk count small
    pk = O.uniform_keys(5, 0, n_probe, 2 * n)
    pk[::97] = hot  # the long chain, hit
    keys = torch.from_numpy(pk).to(DEV)
    want = table.probe(keys, 2048)
    got = table.probe_ordered(keys, 2048)
    torch.cuda.synchronize()
    assert int(got["status"].item()) == 0 and int(want["status"].item()) == 0 and not got.get("exact_retry")
    for k in ("count", "rounds", "round_counts"):
        assert torch.equal(got[k], want[k]), k
    cap = want["cap"]
    valid = (torch.arange(cap, device=DEV)[None, :] < want["count"].to(torch.int64)[:, None]).reshape(-1)
    assert torch.equal(got["sel"][valid], want["sel"][valid])
    assert torch.equal(got["payload"][valid], want["payload"][valid])
    mult = np.where(pk == hot, 299, (pk < n).astype(np.int64))
    rows = np.repeat(np.arange(n_probe, dtype=np.uint64), mult)
    exp = (int(mult.sum()), O.l2_sum(rows, np.repeat(pk, mult)))
    assert ccj.result_checksum(want, 2048) == exp
    pout = table.probe_partitioned(keys, 2048)
    torch.cuda.synchronize()
    assert int(pout["status"].item()) == 0
    assert ccj.result_checksum(pout, 2048, row_map=pout["row_map"].to(torch.int64)) == exp
