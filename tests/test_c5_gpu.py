"""C5: wide payload — 8 int64 build-side payload columns gathered on every match.

Payload of build tuple r, column c: fmix64(r * 8 + c) (distinct per build tuple, so a gather from
the wrong duplicate is caught).  Reference-order tables: every match's table position and payload
row equal the oracle's (L3).  Device-built LP tables: every match's gathered row belongs to a
build tuple with the probe's key, each build tuple at most once per probe row (L2)."""
import numpy as np
import pytest

from helpers import ref_keys
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

P = 8


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


def payload_rows(n):
    r = np.arange(n, dtype=np.uint64)[:, None] * np.uint64(P) + np.arange(P, dtype=np.uint64)[None, :]
    return O.fmix64(r).view(np.int64)


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
@pytest.mark.parametrize("cf", [1, 3])
def test_c5_reference_layout(kind, cf):
    n_build, n_probe, chunk = 1 << 18, 1 << 20, 2048
    bkeys = ref_keys(n_build, cf)
    pay = payload_rows(n_build)
    table = ccj.Table.from_host(kind, bkeys)
    table.set_payload(torch.from_numpy(pay.reshape(-1)).cuda(), P)
    keys = O.uniform_keys(123 + cf, 0, n_probe, n_build + n_build // 4)
    out = table.probe(torch.from_numpy(keys).cuda(), chunk, pos=True, payload_cols=P)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    otab = O.Table(kind, bkeys)
    want = otab.probe(keys, chunk, cap_factor=cf, max_rounds=out["max_rounds"])
    cnt = out["count"].cpu().numpy()
    assert np.array_equal(cnt.view(np.uint32), want["count"])
    cap = out["cap"]
    valid = (np.arange(cap)[None, :] < cnt[:, None]).reshape(-1)
    gpos = out["pos"].cpu().numpy().view(np.uint32)[valid]
    assert np.array_equal(gpos, want["pos"][valid])
    rows = otab.rows[gpos]
    for c in range(P):
        got = out["payload_cols"][c].cpu().numpy()[valid]
        assert np.array_equal(got, pay[rows, c]), f"payload column {c}"


def test_c5_device_built_lp():
    n_build, n_probe, chunk, cf = 1 << 18, 1 << 20, 2048, 2
    bkeys = ref_keys(n_build, cf)
    pay = payload_rows(n_build)
    table = ccj.Table.on_device(ccj.LP, torch.from_numpy(bkeys).cuda())
    table.set_payload(torch.from_numpy(pay.reshape(-1)).cuda(), P)
    keys = O.uniform_keys(9, 0, n_probe, n_build)
    out = table.probe(torch.from_numpy(keys).cuda(), chunk, pos=True, payload_cols=P)
    torch.cuda.synchronize()
    cnt = out["count"].cpu().numpy().astype(np.int64)
    cap = out["cap"]
    valid = (np.arange(cap)[None, :] < cnt[:, None]).reshape(-1)
    sel = out["sel"].cpu().numpy().view(np.uint32)[valid].astype(np.int64)
    chunk_of = np.repeat(np.arange(len(cnt)), cnt)
    prow = chunk_of * chunk + sel
    col0 = out["payload_cols"][0].cpu().numpy()[valid]
    inv = {int(v): r for r, v in enumerate(pay[:, 0])}
    brow = np.array([inv[int(v)] for v in col0], np.int64)
    assert np.array_equal(bkeys[brow], keys[prow])  # the gathered build tuple has the probe's key
    for c in range(1, P):
        assert np.array_equal(out["payload_cols"][c].cpu().numpy()[valid], pay[brow, c])
    pairs = prow * n_build + brow
    assert len(np.unique(pairs)) == len(pairs)  # each build duplicate gathered once per probe row
    m, _ = O.count_uniform(9, 0, n_probe, n_build, n_build, cf)
    assert len(brow) == m


@pytest.mark.parametrize("cf", [1, 2])
def test_c5_partitioned(cf):
    """C5 on the slot-partitioned path: the walk records every match's table position and the
    gather pass materialises the 8 payload columns; every gathered row belongs to a build tuple
    with the probe row's key, each build tuple once per probe row, and the counts are exact."""
    n_build, n_probe, chunk = 1 << 18, 1 << 20, 2048
    bkeys = ref_keys(n_build, cf)
    pay = payload_rows(n_build)
    table = ccj.Table.on_device(ccj.LP, torch.from_numpy(bkeys).cuda())
    table.set_payload(torch.from_numpy(pay.reshape(-1)).cuda(), P)
    keys = O.uniform_keys(21 + cf, 0, n_probe, n_build + n_build // 8)
    out = table.probe_partitioned(torch.from_numpy(keys).cuda(), chunk, pos=True, payload_cols=P)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    nc, cap = out["n_chunks"], out["cap"]
    cnt = out["count"].cpu().numpy()[:nc].astype(np.int64)
    valid = (np.arange(cap)[None, :] < cnt[:, None]).reshape(-1)
    sel = out["sel"].cpu().numpy()[:nc * cap].view(np.uint32)[valid].astype(np.int64)
    chunk_of = np.repeat(np.arange(nc), cnt)
    prow = out["row_map"].cpu().numpy().view(np.uint32)[chunk_of * chunk + sel].astype(np.int64)
    col0 = out["payload_cols"][0].cpu().numpy()[:nc * cap][valid]
    inv = {int(v): r for r, v in enumerate(pay[:, 0])}
    brow = np.array([inv[int(v)] for v in col0], np.int64)
    assert np.array_equal(bkeys[brow], keys[prow])
    for c in range(1, P):
        assert np.array_equal(out["payload_cols"][c].cpu().numpy()[:nc * cap][valid], pay[brow, c])
    pairs = prow * n_build + brow
    assert len(np.unique(pairs)) == len(pairs)
    m, _ = O.count_uniform(21 + cf, 0, n_probe, n_build + n_build // 8, n_build, cf)
    assert len(brow) == m


@pytest.mark.parametrize("chunk,n_probe,spread", [(2048, 1 << 20, 8), (2048, (1 << 20) + 777, 0), (1000, 1 << 20, 8),
                                                  (1022, 300001, 8), (2048, 1 << 20, 1), (1001, 300001, 8),
                                                  (2048, 3 * 2048 + 5, 0)])
def test_c5_partitioned_rows(chunk, n_probe, spread):
    """C5 under CCJ_PART_ROWS (distinct build keys, the bench's C5 route): the split writes every
    position's row and key into the outputs, probe_walk1<POS> leaves each match's table position at
    its output slot (all-matched chunks) or compacts the chunk (chunks with a miss), the gather reads
    them.  spread: probe keys from [0, n_build + n_build / spread) (0: every probe hits; 1: half
    miss).  sel is the original row; every gathered row belongs to the build tuple with the row's
    key, the payload column holds the key, and the count is exact.  Even chunks take the gather
    with stores transposed through LDS (gather_payload_cols, 512-row steps: 1000 / 1022 / 3 x 2048
    + 5 end in partial steps and odd row counts), an odd chunk (1001) the quad form."""
    n_build = 1 << 18
    bkeys = ref_keys(n_build, 1)
    pay = payload_rows(n_build)
    table = ccj.Table.on_device(ccj.LP, torch.from_numpy(bkeys).cuda())
    table.set_payload(torch.from_numpy(pay.reshape(-1)).cuda(), P)
    assert int(table.max_dup) <= 1
    rng = n_build + (n_build // spread if spread else 0)
    keys = O.uniform_keys(77 + spread, 0, n_probe, rng)
    out = table.probe_partitioned(torch.from_numpy(keys).cuda(), chunk, pos=True, payload_cols=P, rows=True)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0
    nc, cap = out["n_chunks"], out["cap"]
    assert cap == chunk
    cnt = out["count"].cpu().numpy()[:nc].astype(np.int64)
    valid = (np.arange(cap)[None, :] < cnt[:, None]).reshape(-1)
    prow = out["sel"].cpu().numpy()[:nc * cap].view(np.uint32)[valid].astype(np.int64)  # original rows
    assert np.array_equal(out["payload"].cpu().numpy()[:nc * cap][valid], keys[prow])
    col0 = out["payload_cols"][0].cpu().numpy()[:nc * cap][valid]
    inv = {int(v): r for r, v in enumerate(pay[:, 0])}
    brow = np.array([inv.get(int(v), -1) for v in col0], np.int64)
    assert (brow >= 0).all()
    assert np.array_equal(bkeys[brow], keys[prow])
    for c in range(1, P):
        assert np.array_equal(out["payload_cols"][c].cpu().numpy()[:nc * cap][valid], pay[brow, c])
    assert len(np.unique(prow)) == len(prow)  # distinct keys: one match per probe row at most
    m, _ = O.count_uniform(77 + spread, 0, n_probe, rng, n_build, 1)
    assert len(prow) == m


@pytest.mark.parametrize("chunk,n_probe,spread,before_payload", [(2048, 1 << 22, 8, False), (2048, (1 << 22) + 777, 0, False),
                                                                 (1000, 3000001, 8, False), (2048, 1 << 22, 2, True),
                                                                 (1001, 3000001, 8, False), (2048, 1 << 22, -1, False)])
def test_c5_partitioned_rows_slab_order(chunk, n_probe, spread, before_payload):
    """C5 with >= 8 partitions (2^20 build keys: 2^22 slots, 8 windows): the walk writes each chunk's
    matches in order of their slot's sub-range (walk_emit_pos_sub) and the gather takes one slab of
    payload rows per XCD at a time (gather_payload_cols_sub).  Within every chunk the positions'
    sub-ranges never decrease; sel / payload / positions / every payload column stay consistent,
    each probe row once, the count exact.  before_payload: the workspace was sized before the
    payload columns existed (no room for the sub-range starts): row order and the row-order gather.
    An odd chunk (1001) keeps row order (the 16-byte column pairs need an even capacity); spread -1:
    every 16th probe on one key, so the split's overflow area holds that partition's extra runs (its
    chunks are gathered whole, after the slabs)."""
    n_build = 1 << 20
    bkeys = ref_keys(n_build, 1)
    pay = payload_rows(n_build)
    table = ccj.Table.on_device(ccj.LP, torch.from_numpy(bkeys).cuda())
    assert table.size == 1 << 22
    rng = n_build + (n_build // spread if spread > 0 else 0)
    keys_np = O.uniform_keys(91 + spread, 0, n_probe, rng)
    if spread < 0:  # skew: every 16th probe on one key, so its partition's runs overflow into the area
        keys_np[::16] = 5
    keys = torch.from_numpy(keys_np).cuda()
    part = table.alloc_partitioned(n_probe, chunk) if before_payload else None
    table.set_payload(torch.from_numpy(pay.reshape(-1)).cuda(), P)
    out = table.probe_partitioned(keys, chunk, pos=True, payload_cols=P, rows=True, part=part)
    torch.cuda.synchronize()
    kern = ccj.last_gather_kernel()
    slab = not before_payload and chunk % 2 == 0
    assert kern.startswith("gather_payload_cols_sub<8>" if slab else "gather_payload_cols<8>" if chunk % 2 == 0
                           else "gather_payload_quad"), kern
    assert int(out["status"].item()) == 0
    nc, cap = out["n_chunks"], out["cap"]
    cnt = out["count"].cpu().numpy()[:nc].astype(np.int64)
    valid2 = np.arange(cap)[None, :] < cnt[:, None]
    valid = valid2.reshape(-1)
    pos = out["pos"].cpu().numpy()[:nc * cap].view(np.uint32).reshape(nc, cap).astype(np.int64)
    if slab:  # sub-range order inside each chunk (window bits 19: sub-range = bits 16-18)
        sub = (pos >> 16) & 7
        sub = np.where(valid2, sub, 8)
        assert (np.diff(sub, axis=1)[:, :] >= 0)[valid2[:, 1:]].all()
    prow = out["sel"].cpu().numpy()[:nc * cap].view(np.uint32)[valid].astype(np.int64)
    keys_h = keys.cpu().numpy()
    assert np.array_equal(out["payload"].cpu().numpy()[:nc * cap][valid], keys_h[prow])
    assert np.array_equal(table_slots(table)[pos.reshape(-1)[valid]], keys_h[prow])
    col0 = out["payload_cols"][0].cpu().numpy()[:nc * cap][valid]
    order = np.argsort(pay[:, 0])
    at = np.searchsorted(pay[order, 0], col0)
    assert (at < n_build).all() and np.array_equal(pay[order[np.minimum(at, n_build - 1)], 0], col0)
    brow = order[at]
    assert np.array_equal(bkeys[brow], keys_h[prow])
    for c in range(1, P):
        assert np.array_equal(out["payload_cols"][c].cpu().numpy()[:nc * cap][valid], pay[brow, c])
    assert len(np.unique(prow)) == len(prow)
    if spread >= 0:
        m, _ = O.count_uniform(91 + spread, 0, n_probe, rng, n_build, 1)
    else:  # reference keys 0 .. n_build - 1 (cf 1): a probe hits iff its key is below n_build
        m = int((keys_np < n_build).sum())
    assert len(prow) == m


def table_slots(table):
    return table.arrays()["table"]
