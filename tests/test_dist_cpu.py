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
    sc = np.zeros(world, np.int64)
    for d in range(world):  # what ccj_partition_by_owner_grouped writes with self_last = rank (one sub-segment)
        idx = np.nonzero(owner == d)[0]
        s = ccj_dist.slot_of(d, rank, world)
        sk[s * cap:s * cap + len(idx)] = keys[idx]
        sr[s * cap:s * cap + len(idx)] = idx
        sc[s] = len(idx)
    rk, rr, rc = torch.full((world * cap,), -5, dtype=torch.int64), torch.empty(world * cap, dtype=torch.int32), \
        torch.empty(world, dtype=torch.int64)
    ccj_dist.exchange_fixed(torch.from_numpy(sk), torch.from_numpy(sr), torch.from_numpy(sc), rk, rr, rc, world, rank,
                            cap, 1, lambda dst, src: dst.copy_(src))
    # the own segment was copied locally: the receive's last slot is this rank's send slot, bit for bit
    assert np.array_equal(rk[(world - 1) * cap:].numpy(), sk[(world - 1) * cap:])
    build = O.ref_build_keys(n_build, cf)
    t = O.Table(O.LP, build[np_owner(build, world) == rank])
    m, l2 = 0, 0
    for s in range(world):  # receive slot s came from rank src: global row = src * n_probe + local
        src = [d for d in range(world) if ccj_dist.slot_of(d, rank, world) == s][0]
        n = int(rc[s])
        seg_k = rk[s * cap:s * cap + n].numpy()
        assert (np_owner(seg_k, world) == rank).all()
        rows = src * n_probe + rr[s * cap:s * cap + n].numpy().astype(np.int64)
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
    """The pipelined protocol's exchange (fixed-capacity segments, equal splits to the peers, the
    own segment copied locally, u32 local rows, source rank implied by the slot) gives the exact
    membership answer (L1 + L2)."""
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


# ---- the pipelined ShardedProbe protocol itself, on CPU: same class, oracle-backed kernels ----

class HostOps:
    """ccj_dist's ops interface on CPU tensors: numpy stand-ins for the owner split, the segment
    chunk counts and the slot-partitioned local probe (a permuted layout with a row map, probed
    by the oracle).  `local_overflow` makes this rank's local probe raise the slot-split overflow
    flag (ccj.FLAG_PART_OVERFLOW), as the one-pass split does under skew."""

    def __init__(self, local_overflow=False, subs=1):
        import ccj_dist
        self.base = ccj_dist.HostOpsBase()
        self.local_overflow = local_overflow
        self.subs = subs  # sub-segments per destination (the device's grouped partition: 8)
        self.probes = 0

    def __getattr__(self, name):
        return getattr(self.base, name)

    def build_local(self, n_build_total, cf, world, rank, stream):
        from oracle import oracle as O
        build = O.ref_build_keys(n_build_total, cf)
        own = build[np_owner(build, world) == rank]
        self.table, self.cf = O.Table(O.LP, own), cf
        return len(own)

    def fixed_partitioner(self, n, world, sub_cap, self_last):
        import ccj_dist
        S = self.subs

        def run(keys, row_base, sk, sr, sc, status, stream):
            k = keys.numpy()
            owner = np_owner(k, world)
            grp = (np.arange(len(k)) * S) // max(len(k), 1)  # sub-segment g: the g-th 1/S of the batch
            for d in range(world):
                for g in range(S):
                    idx = np.nonzero((owner == d) & (grp == g))[0]
                    seg = ccj_dist.slot_of(d, self_last, world) * S + g  # the own rank's region last
                    sc[seg] = len(idx)
                    keep = idx[:sub_cap]
                    sk[seg * sub_cap:seg * sub_cap + len(keep)] = torch.from_numpy(k[keep])
                    sr[seg * sub_cap:seg * sub_cap + len(keep)] = torch.from_numpy((row_base + keep).astype(np.int32))
                    if len(idx) > sub_cap:
                        status |= 8  # CCJ_FLAG_PART_OVERFLOW, as the device's grouped partition
        return run

    def segment_chunk_counts(self, seg_counts, seg_cap, chunk, out, status, stream):
        per = seg_cap // chunk
        for g, live in enumerate(seg_counts.tolist()):
            if live > seg_cap:
                status |= 1
                live = seg_cap
            for j in range(per):
                out[g * per + j] = max(0, min(chunk, live - j * chunk))

    def alloc_group(self, gslots, chunk, status):
        return {"row_map": None}, {"status": status}

    def probe_group(self, keys, counts, part, out, chunk, stream):
        """Live rows permuted by home slot (the slot split's layout), probed chunk by chunk."""
        from oracle import oracle as O
        self.probes += 1
        k, cnt = keys.numpy(), counts.numpy()
        live = np.concatenate([c * chunk + np.arange(int(n)) for c, n in enumerate(cnt)] + [np.zeros(0, np.int64)])
        order = live[np.argsort(O_hash(k[live]) & np.uint64(self.table.size - 1), kind="stable")]
        part["row_map"] = order
        n = len(order)
        new_counts = np.array([min(chunk, n - c * chunk) for c in range(-(-n // chunk))], np.uint32)
        res = self.table.probe(k[order], chunk, counts=new_counts if n else None, cap_factor=self.cf, max_rounds=4096)
        out.update(count=res["count"], sel=res["sel"], payload=res["payload"], cap=res["cap"])
        if self.local_overflow:
            out["status"] |= 8  # CCJ_FLAG_PART_OVERFLOW

    def group_rows(self, part, recv_rows, n_probe, seg_cap, slots, stream, src):
        q = np.arange(recv_rows.numel()) % slots
        recv = np.asarray(src, np.int64)[q // seg_cap] * n_probe + recv_rows.numpy().astype(np.int64)
        return recv[part["row_map"]]

    def checksum(self, out, chunk, row_map, stream):
        from oracle import oracle as O
        rm = row_map.numpy() if isinstance(row_map, torch.Tensor) else row_map
        m, l2 = 0, 0
        for c in range(len(out["count"])):
            k = int(out["count"][c])
            sel = out["sel"][c * out["cap"]:c * out["cap"] + k].astype(np.int64)
            m += k
            l2 = (l2 + O.l2_sum(rm[c * chunk + sel].astype(np.uint64), out["payload"][c * out["cap"]:c * out["cap"] + k])) \
                % (1 << 64)
        return m, l2

    def owner_partitioner(self, n, world):
        def run(keys, row_base, stream):
            k = keys.numpy()
            owner = np_owner(k, world)
            order = np.argsort(owner, kind="stable")
            return (torch.from_numpy(k[order]), torch.from_numpy(row_base + order.astype(np.int64)),
                    torch.from_numpy(np.bincount(owner, minlength=world).astype(np.int64)))
        return run

    def probe_exact(self, keys, chunk, stream):
        res = self.table.probe(keys.numpy(), chunk, cap_factor=self.cf, max_rounds=4096)
        return dict(count=res["count"], sel=res["sel"], payload=res["payload"], cap=res["cap"])


def O_hash(k):
    return np_hash(k)


def _sharded_worker(rank, world, port, cfg, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "chunk-compaction-in-vectorized-execution-simd_amd"),
                    os.path.join(root, "tests")]
    from oracle import oracle as O
    import ccj_dist
    from test_dist_cpu import HostOps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_build, cf, n_probe, rng, seed, chunk, batches, group, skew_rank, local_ovf_rank, subs = cfg[:11]
    run_steps = cfg[11] if len(cfg) > 11 else 0  # > 0: one pipelined run of that many steps
    ops = HostOps(local_overflow=(rank == local_ovf_rank), subs=subs)
    sp = ccj_dist.ShardedProbe(n_build, cf, n_probe, chunk, world, rank, batches=batches, ops=ops, group=group)
    keys = O.uniform_keys(seed, rank * n_probe, (rank + 1) * n_probe, rng)
    if rank == skew_rank:  # one hot key: its owner's send segment overflows on this rank only
        keys[:] = keys[0]
    res = []
    if run_steps:
        m, l2 = sp.run(torch.from_numpy(keys), rank * n_probe, steps=run_steps, verify=True)
        res.append((m, l2, sp.last_exact))
    for _ in range(0 if run_steps else 2):
        m, l2 = sp.step(torch.from_numpy(keys), rank * n_probe, verify=True)
        res.append((m, l2, sp.last_exact))
    probes_verified = ops.probes
    if not run_steps and not sp.last_exact:
        # a timed (verify=False) step moves counts and keys only: the received rows stay as they were
        # (poisoned here) and every local probe's result is the verify step's
        used = [o for o in sp.outs if "count" in o]  # (one group per step: one receive-group slot in use)
        before = [dict(count=o["count"].copy(), payload=o["payload"].copy()) for o in used]
        for rr in sp.rr:
            rr.fill_(-7)
        sp.step(torch.from_numpy(keys), rank * n_probe, verify=False)
        assert all(bool((rr == -7).all()) for rr in sp.rr), "rows crossed in a timed step"
        for b, o in zip(before, used):
            assert np.array_equal(b["count"], o["count"]) and np.array_equal(b["payload"], o["payload"])
    tot = torch.tensor([m, l2 - (1 << 64) if l2 >= (1 << 63) else l2], dtype=torch.int64)
    dist.all_reduce(tot)
    # the exact answer for this rank's stream (full build side, global rows)
    want = O.Table(O.LP, O.ref_build_keys(n_build, cf)).probe_totals(keys, chunk, row_base=rank * n_probe)
    wt = torch.tensor([want[0], want[1] - (1 << 64) if want[1] >= (1 << 63) else want[1]], dtype=torch.int64)
    dist.all_reduce(wt)
    q.put((rank, int(tot[0]), int(tot[1]) % (1 << 64), int(wt[0]), int(wt[1]) % (1 << 64),
           [r[2] for r in res], sp.batches, sp.n_groups, probes_verified))
    dist.destroy_process_group()


def _run_sharded(world, cfg, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = sorted(q.get(timeout=timeout) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():  # a diverged collective sequence hangs: never leave it running
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    return got


@pytest.mark.parametrize("world,batches,group,subs", [(2, 3, 2, 1), (2, 4, 8, 1), (4, 5, 2, 1), (2, 3, 2, 8),
                                                       (4, 5, 2, 8)])
def test_sharded_probe_protocol_gloo(world, batches, group, subs):
    """ShardedProbe.step end to end with gloo: batching, double-buffered send slots, receive-group
    slots (short last group included), group_row_map and the verify checksum; L1 + L2 equal the
    exact answer over all ranks' streams and no rank falls back.  subs = 8: every destination's
    region in 8 sub-segments, as the device's one-pass grouped owner partition writes it."""
    cfg = (1 << 13, 2, 3 << 12, 3 << 12, 21, 256, batches, group, -1, -1, subs)
    got = _run_sharded(world, cfg)
    for rank, m, l2, wm, wl2, exact, nb, ng, probes in got:
        assert (m, l2) == (wm, wl2)
        assert exact == [False, False]
        assert nb == batches and ng == -(-batches // min(batches, group)) and probes == 2 * ng


@pytest.mark.parametrize("world,skew_rank,local_ovf_rank,subs", [(2, 0, -1, 1), (2, -1, 1, 1), (4, 2, -1, 1),
                                                                  (2, 0, -1, 8)])
def test_sharded_overflow_on_one_rank_all_fall_back(world, skew_rank, local_ovf_rank, subs):
    """An overflow seen by ONE rank only (a hot key overflowing its send segment, or the local
    probe's slot split overflowing) makes EVERY rank redo the step with the exact-size protocol:
    the status word is all-reduced before the branch, so no collective sequence diverges (a hang
    here is caught by the queue timeout).  Results stay exact."""
    # subs = 8: one batch, so the hot key's rows (1/8 of the batch per sub-segment) exceed sub_cap
    batches, group = (3, 2) if subs == 1 else (1, 1)
    cfg = (1 << 13, 2, 3 << 12, 3 << 12, 22, 256, batches, group, skew_rank, local_ovf_rank, subs)
    got = _run_sharded(world, cfg)
    for rank, m, l2, wm, wl2, exact, nb, ng, probes in got:
        assert (m, l2) == (wm, wl2)
        assert exact == [True, True]


@pytest.mark.parametrize("world,batches,group,subs,steps,skew_rank", [(2, 3, 2, 1, 3, -1), (2, 4, 3, 8, 2, -1),
                                                                       (4, 5, 2, 1, 2, -1), (2, 3, 2, 1, 2, 1)])
def test_sharded_run_pipelined_steps_gloo(world, batches, group, subs, steps, skew_rank):
    """ShardedProbe.run: `steps` passes issued back to back (the receive-group slots alternate across
    step boundaries, odd group counts included; one status agreement at the end): L1 + L2 are
    `steps` times one pass's exact answer, and an overflow on one rank makes every rank redo all
    the run's steps exactly."""
    cfg = (1 << 13, 2, 3 << 12, 3 << 12, 23, 256, batches, group, skew_rank, -1, subs, steps)
    got = _run_sharded(world, cfg)
    for rank, m, l2, wm, wl2, exact, nb, ng, probes in got:
        assert (m, l2) == (steps * wm, steps * wl2 % (1 << 64))
        assert exact == [skew_rank >= 0]
        if skew_rank < 0:
            assert probes == steps * ng


def _timed_resolve_worker(rank, world, port, cfg, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "chunk-compaction-in-vectorized-execution-simd_amd"),
                    os.path.join(root, "tests")]
    from oracle import oracle as O
    import ccj_dist
    from test_dist_cpu import HostOps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_build, cf, n_probe, rng, seed, chunk, batches, group, subs, steps = cfg
    ops = HostOps(subs=subs)
    sp = ccj_dist.ShardedProbe(n_build, cf, n_probe, chunk, world, rank, batches=batches, ops=ops, group=group, keep_rows=True)
    keys = O.uniform_keys(seed, rank * n_probe, (rank + 1) * n_probe, rng)
    for rr in sp.rr:
        rr.fill_(-7)  # poisoned: a timed run moves no rows
    sp.run(torch.from_numpy(keys), rank * n_probe, steps=steps, timing=True)
    assert not sp.last_exact
    assert all(bool((rr == -7).all()) for rr in sp.rr), "rows crossed in a timed run"
    m, l2, covered = sp.resolve_kept_groups()
    tot = torch.tensor([m, l2 - (1 << 64) if l2 >= (1 << 63) else l2], dtype=torch.int64)
    dist.all_reduce(tot)
    # the exact answer over the covered batches' rows of EVERY source rank (this rank's share here)
    table = O.Table(O.LP, O.ref_build_keys(n_build, cf))
    wm, wl2 = 0, 0
    for i in covered:
        lo, n = sp._batch(i)
        a, b = table.probe_totals(keys[lo:lo + n], chunk, row_base=rank * n_probe + lo)
        wm, wl2 = wm + a, (wl2 + b) % (1 << 64)
    wt = torch.tensor([wm, wl2 - (1 << 64) if wl2 >= (1 << 63) else wl2], dtype=torch.int64)
    dist.all_reduce(wt)
    q.put((rank, int(tot[0]), int(tot[1]) % (1 << 64), int(wt[0]), int(wt[1]) % (1 << 64), sorted(covered)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,batches,group,subs,steps", [(2, 5, 2, 1, 1), (2, 4, 1, 8, 2), (4, 3, 4, 1, 2)])
def test_sharded_timed_run_rows_resolvable_gloo(world, batches, group, subs, steps):
    """a timed run moves keys only (8 B per tuple), so its matches must stay traceable to
    their probe rows through the senders' kept row buffers (one per batch).  After a timed run the
    groups whose results are still held (the last two) get their rows by an untimed all-to-all of
    those buffers, and their L1 + L2 over GLOBAL rows equal the exact answer for those batches on
    every source rank; no row crossed during the run."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    cfg = (1 << 13, 2, 3 << 12, 3 << 12, 31, 256, batches, group, subs, steps)
    procs = [ctx.Process(target=_timed_resolve_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        got = sorted(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for p in procs:
        assert p.exitcode == 0
    n_groups = -(-batches // group)
    want_cov = sorted(range(max(0, n_groups - 2) * group, batches))
    for rank, m, l2, wm, wl2, covered in got:
        assert (m, l2) == (wm, wl2) and m > 0
        assert covered == want_cov
