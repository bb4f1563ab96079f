"""C3: chaining table + compactor under Zipf-skewed probe keys with ~10% match rate
(the selection-vector-pack stress case), at a size the oracle finishes in seconds.

Workload (seeded, numpy): hit w.p. 0.10 -> build_key[pi(zipf_rank)], Zipf s = 1.0 over the build
ranks, pi a fixed hash permutation; miss -> uniform in [2^40, 2^62) (never a build key).
Parity: probe at L3 against the oracle (chaining layout = reference insertion order), compaction
against the sequential compactor simulation, L1 against the hit count."""
import numpy as np
import pytest

from helpers import ref_keys, views_from_rounds, assert_trace_equal
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402
from test_compact_gpu import expected_compaction  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


def zipf_keys(build_keys, n, seed, hit=0.10, s=1.0):
    rng = np.random.default_rng(seed)
    m = len(build_keys)
    ranks = np.arange(1, m + 1, dtype=np.float64)
    cdf = np.cumsum(ranks ** -s)
    cdf /= cdf[-1]
    r = np.searchsorted(cdf, rng.random(n), side="right")
    perm = np.argsort(O.fmix64(np.arange(m, dtype=np.uint64) + np.uint64(seed)))
    keys = build_keys[perm[np.minimum(r, m - 1)]]
    is_hit = rng.random(n) < hit
    miss = rng.integers(1 << 40, 1 << 62, size=n, dtype=np.int64)
    return np.where(is_hit, keys, miss), is_hit


@pytest.mark.parametrize("cf,chunk", [(1, 2048), (2, 2048), (1, 256)])
def test_c3_chaining_zipf_probe_and_compact(cf, chunk):
    n_build, n_probe = 1 << 20, 1 << 22
    bkeys = ref_keys(n_build, cf)
    keys, is_hit = zipf_keys(np.unique(bkeys), n_probe, seed=42 + cf)
    table = ccj.Table.from_host(ccj.CHAIN, bkeys)
    dkeys = torch.from_numpy(keys).cuda()
    out = table.probe(dkeys, chunk)
    comp = ccj.compact(out, chunk, cols=[dkeys])
    torch.cuda.synchronize()
    assert int(out["status"].item()) == 0 and int(comp["status"].item()) == 0
    ores = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}
    ores["sel"] = ores["sel"].view(np.uint32)
    # L1: every hit matches cf times, misses never
    assert int(ores["count"].sum()) == int(is_hit.sum()) * cf
    rate = is_hit.mean()
    assert 0.09 < rate < 0.11
    # L3 vs oracle (both Next views)
    want = O.Table(O.CHAIN, bkeys).probe(keys, chunk, cap_factor=cf, max_rounds=ores["max_rounds"])
    for merged in (False, True):
        g = views_from_rounds(ores["count"], ores["sel"], ores["payload"], ores["rounds"], ores["round_counts"],
                              ores["cap"], ores["max_rounds"], merged=merged)
        w = views_from_rounds(want["count"], want["sel"], want["payload"], want["rounds"], want["round_counts"],
                              want["cap"], want["max_rounds"], merged=merged)
        assert_trace_equal(g, w)
    # compaction in the fixed NaiveCompactor order, with the probe key column carried along
    occ, want_row, want_pay, want_cols, total = expected_compaction(ores, chunk, keys, [keys])
    n_out = int(comp["n"].item())
    assert n_out == len(occ)
    assert (occ[:-1] == chunk).all()
    v = want_row >= 0
    assert np.array_equal(comp["row"].cpu().numpy()[:n_out * chunk][v], want_row[v])
    assert np.array_equal(comp["cols"][0].cpu().numpy()[:n_out * chunk][v], want_cols[0][v])
    assert np.array_equal(comp["payload"].cpu().numpy()[:n_out * chunk][v], want_pay[v])


def test_c3_device_stream_equals_oracle():
    """ccj_gen_c3_keys (device) is the oracle's ccj_c3_key stream, row for row."""
    for n_build, cf, first in ((1 << 26, 1, 0), (100000, 3, 12345), (7, 2, 1 << 40)):
        got = ccj.gen_c3_keys(1 << 18, 42, n_build, cf, first_row=first).cpu().numpy()
        assert np.array_equal(got, O.c3_keys(42, first, first + (1 << 18), n_build, cf))


@pytest.mark.parametrize("n_build,cf", [(1 << 20, 1), (1 << 20, 2)])
def test_c3_probe_and_compact_at_scale(n_build, cf):
    """C3 at 2^24 probes on a device-built chaining table: L1 + L2 against the membership answer,
    and compaction keeps every match."""
    n = 1 << 24
    table = ccj.Table.reference(ccj.CHAIN, n_build, cf, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_c3_keys(n, 42, n_build, cf)
    out = table.probe(keys, 2048)
    m, l2 = ccj.result_checksum(out, 2048)
    assert int(out["status"].item()) == 0
    assert (m, l2) == O.count_c3(42, 0, n, n_build, cf)
    comp = ccj.compact(out, 2048, cols=[keys])
    torch.cuda.synchronize()
    assert int(comp["status"].item()) == 0
    assert int(comp["counts"][:int(comp["n"].item())].to(torch.int64).sum().item()) == m
