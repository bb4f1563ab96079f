"""GPU kernels of the multi-GPU path on one device: the owner multisplit (ccj_partition_by_owner)
against a numpy stable partition, and a P-shard join emulated on one GPU (P tables, each probing
the keys routed to it) against the exact membership answer (L1 + L2)."""
import numpy as np
import pytest

from oracle import oracle as O
from test_dist_cpu import np_owner

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


@pytest.mark.parametrize("parts,n", [(1, 1000), (2, 100000), (4, 8192), (8, 123457), (64, 50000), (8, 0)])
def test_partition_matches_stable_numpy(parts, n):
    keys = O.uniform_keys(parts + 3, 0, n, 1 << 40)
    part = ccj.OwnerPartitioner(n, parts)
    k, r, cnt = part(torch.from_numpy(keys).cuda(), row_base=1000)
    torch.cuda.synchronize()
    owner = np_owner(keys, parts)
    order = np.argsort(owner, kind="stable")
    assert np.array_equal(cnt.cpu().numpy(), np.bincount(owner, minlength=parts))
    assert np.array_equal(k.cpu().numpy()[:n], keys[order])
    assert np.array_equal(r.cpu().numpy()[:n], 1000 + order)


@pytest.mark.parametrize("parts", [2, 4, 8])
def test_sharded_join_on_one_gpu(parts):
    n_build, cf, n_probe, rng, seed = 1 << 20, 2, 1 << 22, 3 << 19, 5
    bkeys = ccj.gen_reference_keys(0, n_build, n_build, cf)
    bp = ccj.OwnerPartitioner(n_build, parts)
    bk, _, bcnt = bp(bkeys)
    probe = ccj.gen_uniform_keys(n_probe, seed, rng)
    pp = ccj.OwnerPartitioner(n_probe, parts)
    pk, pr, pcnt = pp(probe)
    torch.cuda.synchronize()
    bc, pc = bcnt.tolist(), pcnt.tolist()
    m_tot, l2_tot = 0, 0
    for s in range(parts):
        own = bk[sum(bc[:s]):sum(bc[:s + 1])].clone()
        table = ccj.Table.on_device(ccj.LP, own)
        keys = pk[sum(pc[:s]):sum(pc[:s + 1])].clone()
        rows = pr[sum(pc[:s]):sum(pc[:s + 1])].clone()
        out = table.probe(keys, 2048, rounds=False)
        m, l2 = ccj.result_checksum(out, 2048, row_map=rows)
        assert int(out["status"].item()) == 0
        m_tot += m
        l2_tot = (l2_tot + l2) % (1 << 64)
    assert (m_tot, l2_tot) == O.count_uniform(seed, 0, n_probe, rng, n_build, cf)
