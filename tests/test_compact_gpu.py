"""Device compaction (ccj_compact) against the oracle's literal simulation of the fixed
NaiveCompactor (compactor.cpp:5-41 with :36's fresh temp chunk) — L3 order of the compacted stream,
output chunk counts, and the gathered probe-side columns (DataChunk::Append, base.cpp:15-27)."""
import numpy as np
import pytest

from helpers import ref_keys
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


def expected_compaction(ores, chunk, keys, extra, threshold=0):
    """Segments = every round of every chunk in pipeline order; rows concatenated accordingly."""
    cap, mr = ores["cap"], ores["max_rounds"]
    segs, rows, pays = [], [], []
    for c in range(len(ores["count"])):
        n = int(ores["count"][c])
        segs.extend(int(x) for x in ores["round_counts"][c * mr:c * mr + int(ores["rounds"][c])])
        sel = ores["sel"][c * cap:c * cap + n].astype(np.int64)
        rows.append(c * chunk + sel)
        pays.append(ores["payload"][c * cap:c * cap + n])
    rows = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    pays = np.concatenate(pays) if pays else np.zeros(0, np.int64)
    dest, occ = O.compact_plan(np.array(segs, np.uint32), chunk, threshold)
    total = len(rows)
    want_row = np.full(len(occ) * chunk, -1, np.int64)
    want_pay = np.zeros(len(occ) * chunk, np.int64)
    want_row[dest.astype(np.int64)] = rows
    want_pay[dest.astype(np.int64)] = pays
    want_cols = [np.zeros(len(occ) * chunk, np.int64) for _ in extra]
    for w, col in zip(want_cols, extra):
        w[dest.astype(np.int64)] = col[rows]
    return occ, want_row, want_pay, want_cols, total


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
@pytest.mark.parametrize("chunk,n_build,cf,rng", [(4, 64, 1, 64), (8, 512, 2, 600), (64, 4096, 1, 4096),
                                                  (256, 20000, 3, 90000), (2048, 100000, 1, 100000),
                                                  (2048, 100000, 4, 1000000), (1000, 5000, 5, 5000)])
def test_compact_matches_sequential_compactor(kind, chunk, n_build, cf, rng):
    check_compaction(kind, chunk, n_build, cf, rng, 20 * chunk + chunk // 3)


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
def test_compact_many_chunks(kind):
    """4101 probe chunks: the per-chunk offset scans (csrc/ccj_scan.hip) span three 2048-chunk tiles."""
    check_compaction(kind, 4, 512, 2, 600, 4101 * 4 - 1)


def check_compaction(kind, chunk, n_build, cf, rng, n_probe):
    bkeys = ref_keys(n_build, cf)
    keys = O.uniform_keys(5 + chunk, 0, n_probe, rng)
    extra = [O.uniform_keys(77, 0, n_probe, 1 << 40), np.arange(n_probe, dtype=np.int64) * 3 + 1]
    table = ccj.Table.from_host(kind, bkeys)
    dkeys = torch.from_numpy(keys).cuda()
    dext = [torch.from_numpy(e).cuda() for e in extra]
    out = table.probe(dkeys, chunk)
    comp = ccj.compact(out, chunk, cols=[dkeys] + dext)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0 and int(comp["status"].item()) == 0
    ores = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
    ores["sel"] = ores["sel"].view(np.uint32)
    occ, want_row, want_pay, want_cols, total = expected_compaction(ores, chunk, keys, [keys] + extra)
    n_out = int(comp["n"].item())
    assert n_out == len(occ)
    assert np.array_equal(comp["counts"].cpu().numpy()[:n_out].view(np.uint32), occ)
    got_row = comp["row"].cpu().numpy()[:n_out * chunk]
    valid = want_row >= 0
    assert np.array_equal(got_row[valid], want_row[valid])
    assert np.array_equal(comp["payload"].cpu().numpy()[:n_out * chunk][valid], want_pay[valid])
    for g, w in zip(comp["cols"], want_cols):
        assert np.array_equal(g.cpu().numpy()[:n_out * chunk][valid], w[valid])
    # the compacted multiset equals the uncompacted one
    assert valid.sum() == total


def test_compact_full_chunks_bypass():
    # chunk 4, every probe key present once at its home slot most of the time: many full rounds
    bkeys = ref_keys(16, 1)
    keys = O.uniform_keys(3, 0, 800, 20)  # 4 of 20 key values miss: partial and full Next results
    table = ccj.Table.from_host(ccj.LP, bkeys)
    out = table.probe(torch.from_numpy(keys).cuda(), 4)
    comp = ccj.compact(out, 4)
    torch.cuda.synchronize()
    ores = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
    ores["sel"] = ores["sel"].view(np.uint32)
    rc = [int(x) for c in range(len(ores["count"]))
          for x in ores["round_counts"][c * ores["max_rounds"]:c * ores["max_rounds"] + int(ores["rounds"][c])]]
    assert 4 in rc and any(0 < x < 4 for x in rc)  # both kinds of Next result occur
    occ, want_row, _, _, _ = expected_compaction(ores, 4, keys, [])
    n_out = int(comp["n"].item())
    assert n_out == len(occ)
    assert np.array_equal(comp["row"].cpu().numpy()[:n_out * 4][want_row >= 0], want_row[want_row >= 0])


def test_compact_empty():
    table = ccj.Table.from_host(ccj.LP, ref_keys(100, 1))
    keys = np.arange(1000, 2000, dtype=np.int64)  # no key matches
    out = table.probe(torch.from_numpy(keys).cuda(), 256)
    comp = ccj.compact(out, 256)
    torch.cuda.synchronize()
    assert int(comp["n"].item()) == 0


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
@pytest.mark.parametrize("chunk,threshold", [(256, 1), (256, 64), (256, 200), (2048, 512), (64, 63), (100, 0)])
def test_threshold_gated_compaction(kind, chunk, threshold):
    """Results of >= threshold rows pass through as their own (sparse) chunk, smaller ones are
    compacted — the sequential simulation (oracle compact_plan with a threshold) decides every
    row's output slot and every output chunk's count."""
    bkeys = ref_keys(20000, 3)
    n_probe = 30 * chunk + 17
    keys = O.uniform_keys(chunk + threshold, 0, n_probe, 60000)
    table = ccj.Table.from_host(kind, bkeys)
    dkeys = torch.from_numpy(keys).cuda()
    out = table.probe(dkeys, chunk)
    comp = ccj.compact(out, chunk, cols=[dkeys], threshold=threshold)
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0 and int(comp["status"].item()) == 0
    ores = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
    ores["sel"] = ores["sel"].view(np.uint32)
    occ, want_row, want_pay, want_cols, total = expected_compaction(ores, chunk, keys, [keys], threshold)
    n_out = int(comp["n"].item())
    assert n_out == len(occ)
    assert np.array_equal(comp["counts"].cpu().numpy()[:n_out].view(np.uint32), occ)
    valid = want_row >= 0
    assert np.array_equal(comp["row"].cpu().numpy()[:n_out * chunk][valid], want_row[valid])
    assert np.array_equal(comp["payload"].cpu().numpy()[:n_out * chunk][valid], want_pay[valid])
    assert np.array_equal(comp["cols"][0].cpu().numpy()[:n_out * chunk][valid], want_cols[0][valid])
    assert valid.sum() == total


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
@pytest.mark.parametrize("chunk,cf", [(256, 1), (2048, 3), (1000, 2)])
def test_compact_join_key_column_from_payload(kind, chunk, cf):
    """key_cols: the carried join-key column filled from the payload (probe key == build key on
    every match of the equi-join) equals the gathered one row for row; a NULL source column is
    accepted for it, and the other carried columns are still gathered."""
    bkeys = ref_keys(30000, cf)
    n_probe = 40 * chunk + 5
    keys = O.uniform_keys(chunk + cf, 0, n_probe, 45000)
    extra = np.arange(n_probe, dtype=np.int64) * 7 - 3
    table = ccj.Table.from_host(kind, bkeys)
    dkeys, dext = torch.from_numpy(keys).cuda(), torch.from_numpy(extra).cuda()
    out = table.probe(dkeys, chunk)
    g = ccj.compact(out, chunk, cols=[dkeys, dext])
    k = ccj.compact(out, chunk, cols=[dkeys, dext], key_cols=[0])
    z = ccj.compact(out, chunk, cols=[None, dext], key_cols=[0])
    torch.cuda.synchronize()
    n = int(g["n"].item())
    assert n > 0 and int(k["n"].item()) == n and int(z["n"].item()) == n
    cnt = g["counts"][:n].to(torch.int64)
    valid = (torch.arange(chunk, device=cnt.device)[None, :] < cnt[:, None]).reshape(-1)
    for o in (k, z):
        assert int(o["status"].item()) == 0
        for q in range(2):
            assert torch.equal(o["cols"][q][:n * chunk][valid], g["cols"][q][:n * chunk][valid])
        assert torch.equal(o["payload"][:n * chunk][valid], g["payload"][:n * chunk][valid])
