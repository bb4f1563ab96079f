"""CPU model of the rank walk's window index (csrc/ccj_rank.hip), checked against the oracle.

The rank walk replaces the reference's slot-by-slot run walk (linear_probing_ht.cpp:72-80,
:100-110: from the home slot h, every occupied slot until the first empty one is a candidate) by
three arrays built from the finished table — occ (a bit per slot), pre (occupied slots before each
128-slot block) and ckeys (the occupied slots' keys in slot order) — and, per row, L = the occupied
run length from h inside h's 2^19-slot window and r = rank(h), the candidates being ckeys[r, r + L).
Rows whose run reaches the window's end walk the slot array.  This restates those formulas in numpy
exactly as the kernel evaluates them (128-slot block rank, run length by the first zero bit, the
window-end fallback) and checks the per-row match counts give the oracle's L1 + L2 answer on
tables with clusters that cross window ends and wrap the table."""
import numpy as np

from oracle import oracle as O

WBITS = 19


def np_murmur(x):
    x = x.astype(np.uint64)
    c = np.uint64(0xd6e8feb86659fd93)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(32)
        x *= c
        x ^= x >> np.uint64(32)
        x *= c
        x ^= x >> np.uint64(32)
    return x


def build_index(slots):
    """occ bits, pre per 128-slot block, ckeys — the device build (rank_occ + host scan +
    rank_compact_keys)."""
    occ = slots != -1
    blk = occ.reshape(-1, 128).sum(axis=1)
    pre = np.concatenate([[0], np.cumsum(blk)[:-1]]).astype(np.int64)
    ckeys = slots[occ]
    return occ, pre, ckeys


def rank_walk_counts(slots, keys):
    size = len(slots)
    occ, pre, ckeys = build_index(slots)
    W = 1 << WBITS
    home = (np_murmur(keys) & np.uint64(size - 1)).astype(np.int64)
    # rank(h) = pre[h >> 7] + occupied slots of h's 128-slot block below h
    within = np.cumsum(occ.reshape(-1, 128), axis=1) - occ.reshape(-1, 128)
    r = pre[home >> 7] + within.reshape(-1)[home]
    # L = occupied run from h, cut at the window's end (slow rows: the run reaches it)
    zeros = np.nonzero(~occ)[0]
    j = np.searchsorted(zeros, home)
    nz = np.where(j < len(zeros), zeros[np.minimum(j, len(zeros) - 1)], size + zeros[0])
    win_end = (home // W + 1) * W
    slow = nz >= win_end
    L = np.where(slow, 0, nz - home)
    cnt = np.zeros(len(keys), np.int64)
    for t in range(int(L.max()) if len(L) else 0):  # candidate t of every row at once
        m = L > t
        cnt[m] += ckeys[r[m] + t] == keys[m]
    for i in np.nonzero(slow)[0]:  # the slot array from the home slot, wrapping
        s = home[i]
        while slots[s] != -1:
            cnt[i] += slots[s] == keys[i]
            s = (s + 1) & (size - 1)
    return cnt, slow


def test_rank_model_matches_oracle_with_window_crossing_clusters():
    g = np.random.default_rng(5)
    size = 1 << 21  # 2^19 keys -> 2^21 slots: four windows
    cand = np.unique(g.integers(1, 1 << 40, size=1 << 23, dtype=np.int64))
    g.shuffle(cand)
    home = (np_murmur(cand) & np.uint64(size - 1)).astype(np.int64)
    clusters = [cand[(home >= e - 80) & (home < e)][:300] for e in ((1 << 19), (2 << 19), size)]
    rest = np.setdiff1d(cand[:900000], np.concatenate(clusters))
    n_build = 1 << 19
    build = np.concatenate(clusters + [rest[:n_build - 900]])
    g.shuffle(build)
    T = O.Table(O.LP, build)
    assert T.size == size
    probe = np.concatenate([build[:200000], rest[n_build:n_build + 50000]] + clusters)
    g.shuffle(probe)
    cnt, slow = rank_walk_counts(T.table, probe)
    assert slow.sum() > 0  # some runs do leave their window
    assert cnt.max() <= 1
    rows = np.nonzero(cnt)[0].astype(np.uint64)
    assert (len(rows), O.l2_sum(rows, probe[cnt > 0])) == T.probe_totals(probe, 2048)


def test_rank_model_reference_table():
    """The reference generator's table (the C2 shape at 2^20 keys): every probe of [0, n) matches
    once; runs of up to the table's longest are resolved from the index alone or the fallback."""
    n = 1 << 20
    T = O.Table(O.LP, O.ref_build_keys(n, 1))
    keys = O.uniform_keys(13, 0, 1 << 20, 2 * n)
    cnt, _ = rank_walk_counts(T.table, keys)
    rows = np.nonzero(cnt)[0].astype(np.uint64)
    assert (len(rows), O.l2_sum(rows, keys[cnt > 0])) == T.probe_totals(keys, 2048)
