"""The multi-GPU exchange protocol (ccj_dist.exchange) on CPU with the gloo backend, world size 2.

Every rank owner-partitions its probe keys (owner = murmurhash64(k) >> 63), exchanges keys + global
row ids all-to-all, probes what it received against its shard of the build side with the CPU oracle
(standing in for the GPU probe), and the all-reduced match count / L2 checksum must equal the
exact membership answer for the union of all ranks' probe streams (L1 + L2 parity)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def np_hash(x):
    x = np.asarray(x).astype(np.uint64)
    c = np.uint64(0xD6E8FEB86659FD93)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(32)
        x *= c
        x ^= x >> np.uint64(32)
        x *= c
        x ^= x >> np.uint64(32)
    return x


def np_owner(keys, world):
    if world == 1:
        return np.zeros(len(keys), np.int64)
    shift = np.uint64(64 - int(np.log2(world)))
    return (np_hash(keys) >> shift).astype(np.int64)


def _worker(rank, world, port, cfg, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "chunk-compaction-in-vectorized-execution-simd_amd")]
    from oracle import oracle as O
    import ccj_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_build, cf, n_probe, rng, seed = cfg
    keys = O.uniform_keys(seed, rank * n_probe, (rank + 1) * n_probe, rng)
    owner = np_owner(keys, world)
    order = np.argsort(owner, kind="stable")
    rows = rank * n_probe + np.arange(n_probe, dtype=np.int64)
    counts = np.bincount(owner, minlength=world).astype(np.int64)
    rk, rr, rc = ccj_dist.exchange(torch.from_numpy(keys[order]), torch.from_numpy(rows[order]),
                                   torch.from_numpy(counts))
    build = O.ref_build_keys(n_build, cf)
    own = build[np_owner(build, world) == rank]
    rkeys, rrows = rk.numpy(), rr.numpy()
    assert (np_owner(rkeys, world) == rank).all()
    t = O.Table(O.LP, own)
    res = t.probe(rkeys, 2048, cap_factor=cf, max_rounds=4096)
    cap = res["cap"]
    m, l2 = 0, 0
    for c in range(len(res["count"])):
        k = int(res["count"][c])
        sel = res["sel"][c * cap:c * cap + k].astype(np.int64)
        m += k
        l2 = (l2 + O.l2_sum(rrows[c * 2048 + sel].astype(np.uint64), res["payload"][c * cap:c * cap + k])) % (1 << 64)
    tot = torch.tensor([m, l2 - (1 << 64) if l2 >= (1 << 63) else l2], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        q.put((int(tot[0]), int(tot[1]) % (1 << 64), sum(rc)))
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,cfg", [(2, (50000, 2, 40000, 80000, 7)), (2, (30000, 1, 50000, 30000, 8)),
                                       (4, (20000, 3, 10000, 40000, 9))])
def test_exchange_protocol_gloo(world, cfg):
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    m, l2, _ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_build, cf, n_probe, rng, seed = cfg
    want = O.count_uniform(seed, 0, world * n_probe, rng, n_build, cf)
    assert (m, l2) == want


def _fixed_worker(rank, world, port, cfg, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "chunk-compaction-in-vectorized-execution-simd_amd")]
    from oracle import oracle as O
    import ccj_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_build, cf, n_probe, rng, seed = cfg
    keys = O.uniform_keys(seed, rank * n_probe, (rank + 1) * n_probe, rng)
    owner = np_owner(keys, world)
    cap = ccj_dist.seg_capacity(n_probe, world, 2048)
    sk = np.full(world * cap, -1, np.int64)
    sr = np.zeros(world * cap, np.int32)
    sc = np.bincount(owner, minlength=world).astype(np.int64)
    for d in range(world):  # what ccj_partition_by_owner_fixed writes
        idx = np.nonzero(owner == d)[0]
        sk[d * cap:d * cap + len(idx)] = keys[idx]
        sr[d * cap:d * cap + len(idx)] = idx
    rk, rr, rc = torch.empty(world * cap, dtype=torch.int64), torch.empty(world * cap, dtype=torch.int32), \
        torch.empty(world, dtype=torch.int64)
    ccj_dist.exchange_fixed(torch.from_numpy(sk), torch.from_numpy(sr), torch.from_numpy(sc), rk, rr, rc)
    build = O.ref_build_keys(n_build, cf)
    t = O.Table(O.LP, build[np_owner(build, world) == rank])
    m, l2 = 0, 0
    for g in range(world):  # receive segment g came from rank g: global row = g * n_probe + local
        n = int(rc[g])
        seg_k = rk[g * cap:g * cap + n].numpy()
        assert (np_owner(seg_k, world) == rank).all()
        rows = g * n_probe + rr[g * cap:g * cap + n].numpy().astype(np.int64)
        res = t.probe(seg_k, 2048, cap_factor=cf, max_rounds=4096)
        cap_o = res["cap"]
        for c in range(len(res["count"])):
            k = int(res["count"][c])
            sel = res["sel"][c * cap_o:c * cap_o + k].astype(np.int64)
            m += k
            l2 = (l2 + O.l2_sum(rows[c * 2048 + sel].astype(np.uint64), res["payload"][c * cap_o:c * cap_o + k])) \
                % (1 << 64)
    tot = torch.tensor([m, l2 - (1 << 64) if l2 >= (1 << 63) else l2], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        q.put((int(tot[0]), int(tot[1]) % (1 << 64)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_fixed_capacity_exchange_gloo(world):
    """The pipelined protocol's exchange (fixed-capacity segments, equal splits, u32 local rows,
    source rank implied by the segment) gives the exact membership answer (L1 + L2)."""
    from oracle import oracle as O
    cfg = (1 << 14, 2, 1 << 15, 3 << 13, 9)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_fixed_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_build, cf, n_probe, rng, seed = cfg
    assert got == O.count_uniform(seed, 0, world * n_probe, rng, n_build, cf)
