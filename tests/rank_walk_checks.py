"""The rank walk (csrc/ccj_rank.hip): the partitioned LP walk with each table window's occupancy
bitmap + rank in LDS and the candidate keys read from the compact key array.  Built into
libccj_tuning.so only: tests/test_rank_gpu.py runs this file in a child pytest with CCJ_LIB_PATH
naming that library.

Opt-in (CCJ_PART_RANK; DESIGN §3.3 has why it is not the default).  It must give the slot-array
walk's matches — every chunk's stream in row order, every payload its row's key — and the exact
L1 + L2 answer.  Covered: misses
(compacted chunks), rows mode and position mode, chunks of 512 / 1024 / 2048, segmented input
counts, runs that leave their window (and wrap around the table's end) and runs far longer than one
4-key window.  Reference semantics: a row's candidates are the occupied slots from its home slot to
the first empty one (linear_probing_ht.cpp:72-80, :100-110)."""
import numpy as np
import pytest
import torch

import ccj
from oracle import oracle as O

pytestmark = pytest.mark.gpu

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def np_murmur(x):
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


def matches(out, chunk, keys_h):
    """(global rows, payloads) of a partitioned output sorted by row, after checking each chunk's
    stream: in row (position) order, every payload the matched row's key."""
    n = out["n_chunks"]
    cnt = out["count"][:n].cpu().numpy().view(np.uint32).astype(np.int64)
    cap = out["cap"]
    valid = np.arange(cap)[None, :] < cnt[:, None]
    sel = out["sel"][:n * cap].cpu().numpy().view(np.uint32).reshape(n, cap).astype(np.int64)
    pay = out["payload"][:n * cap].cpu().numpy().reshape(n, cap)[valid]
    if out["rows_in_sel"]:
        rows = sel[valid]
    else:  # sel = position in the chunk: strictly increasing inside each chunk
        inc = (sel[:, 1:] > sel[:, :-1]) | ~valid[:, 1:]
        assert bool(inc.all()), "a chunk's matches are not in row order"
        rm = out["row_map"].cpu().numpy().view(np.uint32).astype(np.int64)
        rows = rm[(np.arange(n)[:, None] * chunk + sel)[valid]]
    assert np.array_equal(pay, keys_h[rows]), "a payload is not its row's key"
    o = np.argsort(rows, kind="stable")
    return rows[o], pay[o]


def both_walks(table, keys, chunk, **kw):
    """The rank walk (CCJ_PART_RANK) and the slot-array walk give the same matches.  (The
    one-pass split places runs by atomic reservation, so two calls lay the column out in different
    orders: the comparison is per row, not per position.)"""
    kh = keys.cpu().numpy()
    a = table.probe_partitioned(keys, chunk, rank=True, **kw)
    torch.cuda.synchronize()
    ra, pa = matches(a, chunk, kh)
    b = table.probe_partitioned(keys, chunk, **kw)
    torch.cuda.synchronize()
    rb, pb = matches(b, chunk, kh)
    assert int(a["status"].item()) == 0 and int(b["status"].item()) == 0
    assert not a.get("exact_retry") and not b.get("exact_retry")
    assert np.array_equal(ra, rb) and np.array_equal(pa, pb), "rank walk and slot walk matches differ"
    return table.probe_partitioned(keys, chunk, rank=True, **kw)


@pytest.mark.parametrize("rows", [True, False])
@pytest.mark.parametrize("n_build,n_probe,rng,chunk", [
    (1 << 20, 1 << 22, 1 << 20, 2048),       # every row matches: no chunk is compacted
    (1 << 20, 1 << 22, 3 << 19, 2048),       # 1/3 misses
    (1 << 20, 3000001, 5 << 20, 1024),       # 80 % misses, ragged end
    (1 << 18, 1 << 21, 1 << 18, 512),        # two windows, chunk 512
    (3 << 18, 1 << 21, 1 << 20, 1536),       # chunk 1536 (3 blocks)
])
def test_rank_walk_equals_slot_walk(n_build, n_probe, rng, chunk, rows):
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(n_probe, 53, rng)
    out = both_walks(table, keys, chunk, rows=rows)
    want = O.count_uniform(53, 0, n_probe, rng, n_build, 1)
    if rows:
        assert ccj.result_checksum(out, 0) == want
    else:
        assert ccj.result_checksum(out, chunk, row_map=out["row_map"].to(torch.int64)) == want
    table.free()


def test_rank_walk_runs_leaving_the_window():
    """A host-built (reference-order) table of 2^18 keys = 2^20 slots = two 2^19-slot windows, with
    clusters of keys hashed just below each window's end: their runs cross into the next window
    (and, for the last window, wrap around to slot 0), so the rank walk hands those rows to the
    slot array; the clusters' runs are hundreds of keys long (many 4-key windows per row)."""
    g = np.random.default_rng(11)
    size = 1 << 20
    cand = np.unique(g.integers(1, 1 << 40, size=1 << 24, dtype=np.int64))
    g.shuffle(cand)
    home = (np_murmur(cand.astype(np.uint64)) & np.uint64(size - 1)).astype(np.int64)
    edge0 = cand[(home >= (1 << 19) - 96) & (home < (1 << 19))][:400]
    edge1 = cand[(home >= size - 96)][:400]
    assert len(edge0) == 400 and len(edge1) == 400
    rest = np.setdiff1d(cand[:600000], np.concatenate([edge0, edge1]))
    n_build = 1 << 18
    build = np.concatenate([edge0, edge1, rest[:n_build - 800]])
    g.shuffle(build)
    table = ccj.Table.from_host(ccj.LP, build)
    assert table.size == size
    misses = rest[n_build:n_build + 50000]
    pk = np.concatenate([build, build[:1000], misses, edge0, edge1, edge1])
    g.shuffle(pk)
    keys = torch.from_numpy(pk).cuda()
    for rows in (True, False):
        out = both_walks(table, keys, 2048, rows=rows)
        hit = np.isin(pk, build)
        r = np.nonzero(hit)[0].astype(np.uint64)
        want = (len(r), O.l2_sum(r, pk[hit]))
        if rows:
            assert ccj.result_checksum(out, 0) == want
        else:
            assert ccj.result_checksum(out, 2048, row_map=out["row_map"].to(torch.int64)) == want
    table.free()


def test_rank_walk_segmented_counts():
    """Input chunk counts (the multi-GPU receive buffers): dead rows hold keys that would match."""
    chunk, n_chunks, n_build = 2048, 900, 1 << 20
    g = np.random.default_rng(9)
    keys_h = g.integers(0, 2 * n_build, size=n_chunks * chunk).astype(np.int64)
    counts_h = g.integers(0, chunk + 1, size=n_chunks).astype(np.uint32)
    counts_h[::5] = chunk
    counts_h[2::13] = 0
    table = ccj.Table.reference(ccj.LP, n_build, 1, ccj.LAYOUT_DEVICE)
    counts = torch.from_numpy(counts_h.view(np.int32)).cuda()
    out = both_walks(table, torch.from_numpy(keys_h).cuda(), chunk, counts=counts)
    pos = np.arange(n_chunks * chunk)
    live = ((pos % chunk) < counts_h[pos // chunk]) & (keys_h < n_build)
    want = (int(live.sum()), O.l2_sum(pos[live].astype(np.uint64), keys_h[live]))
    assert ccj.result_checksum(out, chunk, row_map=out["row_map"].to(torch.int64)) == want
    table.free()


def test_rank_walk_needs_the_index():
    """CCJ_PART_RANK on a table without its window index is refused (the index is opt-in, built by
    ccj_table_build_rank_index), not silently replaced by the slot walk."""
    table = ccj.Table.reference(ccj.LP, 1 << 18, 1, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(1 << 20, 3, 1 << 18)
    part = table.alloc_partitioned(keys.numel(), 2048)
    with pytest.raises(ccj.CCJError):
        table.probe_partitioned(keys, 2048, part=part, rank=True)
    table.free()
