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


@pytest.mark.parametrize("parts,n,base", [(1, 1000, 0), (2, 100000, 7), (8, 123457, 1 << 20), (64, 50000, 3)])
def test_partition_fixed_segments(parts, n, base):
    """ccj_partition_by_owner_fixed: segment d holds exactly the owner-d (key, base + row) pairs
    (in any order), and the true counts."""
    from ccj_dist import seg_capacity
    keys = O.uniform_keys(parts + 11, 0, n, 1 << 40)
    cap = seg_capacity(n, parts, 256)
    fp = ccj.FixedOwnerPartitioner(n, parts, cap)
    ok = torch.full((parts * cap,), -7, dtype=torch.int64, device="cuda")
    orow = torch.zeros(parts * cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(parts, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    fp(torch.from_numpy(keys).cuda(), base, ok, orow, cnt, st)
    torch.cuda.synchronize()
    owner = np_owner(keys, parts)
    want_cnt = np.bincount(owner, minlength=parts)
    assert int(st.item()) == 0
    assert np.array_equal(cnt.cpu().numpy(), want_cnt)
    k, r = ok.cpu().numpy(), orow.cpu().numpy()
    for d in range(parts):
        idx = np.nonzero(owner == d)[0]
        gr = r[d * cap:d * cap + len(idx)].astype(np.int64) - base
        assert np.array_equal(np.sort(gr), idx)  # every owner-d row exactly once
        assert np.array_equal(k[d * cap:d * cap + len(idx)], keys[gr])  # each with its own key
        assert (k[d * cap + len(idx):(d + 1) * cap] == -7).all()  # padding untouched


def test_partition_fixed_overflow_flags_and_stays_in_bounds():
    n, parts, cap = 100000, 4, 1024  # far too small: most rows dropped
    keys = O.uniform_keys(1, 0, n, 1 << 40)
    fp = ccj.FixedOwnerPartitioner(n, parts, cap)
    ok = torch.full((parts * cap + 64,), -7, dtype=torch.int64, device="cuda")
    orow = torch.zeros(parts * cap + 64, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(parts, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    fp(torch.from_numpy(keys).cuda(), 0, ok, orow, cnt, st)
    torch.cuda.synchronize()
    assert int(st.item()) & 1
    assert (ok[parts * cap:].cpu().numpy() == -7).all()
    owner = np_owner(keys, parts)
    kk = ok[:parts * cap].cpu().numpy()
    for d in range(parts):  # what was kept of destination d is owner-d keys only, segment full
        assert (np_owner(kk[d * cap:(d + 1) * cap], parts) == d).all()


@pytest.mark.parametrize("parts,n,base,self_last", [(1, 1000, 0, -1), (2, 100000, 7, -1), (8, 1234567, 1 << 20, -1),
                                                    (64, 500000, 3, -1), (1, 1000, 0, 0), (2, 100000, 7, 0),
                                                    (8, 1234567, 1 << 20, 3), (8, 300000, 5, 7), (64, 500000, 3, 17),
                                                    (4, 777777, 11, -1), (4, 200000, 0, 2), (16, 400000, 1, 5),
                                                    (32, 300000, 2, -1)])
def test_partition_grouped_segments(parts, n, base, self_last):
    """ccj_partition_by_owner_grouped (the one-pass split with the owner as partition): the 8
    sub-segments of destination d's slot hold exactly the owner-d (key, base + row) pairs between
    them (in any order), their counts are the true counts, and nothing past a count is written.
    self_last = r: the own rank's region in the last slot, the peers' in rank order before it."""
    G = ccj.OWNER_GROUPS
    keys = O.uniform_keys(parts + 13, 0, n, 1 << 40)
    cap = ccj.grouped_sub_cap(n, parts, 256)
    fp = ccj.GroupedOwnerPartitioner(n, parts, cap, self_last=self_last)
    ok = torch.full((parts * G * cap,), -7, dtype=torch.int64, device="cuda")
    orow = torch.zeros(parts * G * cap, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(parts * G, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    fp(torch.from_numpy(keys).cuda(), base, ok, orow, cnt, st)
    torch.cuda.synchronize()
    owner = np_owner(keys, parts)
    slot = [d if self_last < 0 else (parts - 1 if d == self_last else d - (d > self_last)) for d in range(parts)]
    assert sorted(slot) == list(range(parts))
    c = cnt.cpu().numpy().reshape(parts, G)[slot]  # row d: destination d's sub-segment counts
    assert int(st.item()) == 0
    assert np.array_equal(c.sum(axis=1), np.bincount(owner, minlength=parts))
    k, r = ok.cpu().numpy(), orow.cpu().numpy()
    for d in range(parts):
        rows, ks = [], []
        for g in range(G):
            lo = (slot[d] * G + g) * cap
            rows.append(r[lo:lo + c[d, g]].astype(np.int64) - base)
            ks.append(k[lo:lo + c[d, g]])
            assert (k[lo + c[d, g]:lo + cap] == -7).all()  # padding untouched
        rows, ks = np.concatenate(rows), np.concatenate(ks)
        assert np.array_equal(np.sort(rows), np.nonzero(owner == d)[0])  # every owner-d row exactly once
        assert np.array_equal(ks, keys[rows])  # each with its own key


def test_partition_grouped_overflow_flags_and_stays_in_bounds():
    n, parts, cap = 300000, 4, 1024  # far too small: most rows dropped
    G = ccj.OWNER_GROUPS
    keys = O.uniform_keys(1, 0, n, 1 << 40)
    fp = ccj.GroupedOwnerPartitioner(n, parts, cap)
    ok = torch.full((parts * G * cap + 64,), -7, dtype=torch.int64, device="cuda")
    orow = torch.zeros(parts * G * cap + 64, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(parts * G, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    fp(torch.from_numpy(keys).cuda(), 0, ok, orow, cnt, st)
    torch.cuda.synchronize()
    assert int(st.item()) & ccj.FLAG_PART_OVERFLOW
    assert (ok[parts * G * cap:].cpu().numpy() == -7).all()
    kk = ok[:parts * G * cap].cpu().numpy()
    for d in range(parts):  # what was kept of destination d is owner-d keys only
        seg = kk[d * G * cap:(d + 1) * G * cap]
        assert (np_owner(seg[seg != -7], parts) == d).all()


def test_segment_chunk_counts():
    cap, chunk = 4096, 1024
    cnt = torch.tensor([0, 1, 1024, 1025, 4096, 5000], dtype=torch.int64, device="cuda")
    out = torch.full((len(cnt) * cap // chunk,), 99, dtype=torch.int32, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    ccj.segment_chunk_counts(cnt, cap, chunk, out, st)
    torch.cuda.synchronize()
    want = [0, 0, 0, 0, 1, 0, 0, 0, 1024, 0, 0, 0, 1024, 1, 0, 0, 1024] + [1024] * 7
    assert out.cpu().tolist() == want[:len(want)]
    assert int(st.item()) & 1  # 5000 > cap


@pytest.fixture(scope="module")
def pg1():
    """A one-rank RCCL process group: all-to-all degenerates to a copy, but the streams, events,
    double buffering and the fallback path of ShardedProbe run as they do at N ranks."""
    import os
    import torch.distributed as dist
    from test_dist_cpu import free_port
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


@pytest.mark.parametrize("batches", [1, 3, 4, 20])
def test_sharded_probe_pipelined_one_rank(pg1, batches):
    import ccj_dist
    n_build, n_probe = 1 << 20, 3 << 20
    sp = ccj_dist.ShardedProbe(n_build, 1, n_probe, 2048, 1, 0, batches=batches)
    keys = ccj.gen_uniform_keys(n_probe, 42, n_build + (n_build >> 2))
    want = O.count_uniform(42, 0, n_probe, n_build + (n_build >> 2), n_build, 1)
    for _ in range(2):
        sp.step(keys, 0)
    assert sp.step(keys, 0, verify=True) == want
    assert not sp.last_exact
    # force the overflow fallback: shrink the segment capacity below the batch size
    sp._resize(2048)
    assert sp.step(keys, 0, verify=True) == want
    assert sp.last_exact


def test_bench_sharded_line():
    """bench.py's N > 1 step (bench_multi) end to end on one GPU through bench.py's own launcher
    (--gpus 1 --sharded, no outside torchrun: a one-rank RCCL group in a child process), at a small
    size: exactly one JSON line of the driver's contract with the N > 1 diagnostics, L1 + L2 exact."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--sharded", "--steps", "2", "--warmup", "1",
                        "--no-cpu", "--n-build-per-gpu", str(1 << 22), "--n-probe", str(1 << 24), "--batches", "4"],
                       cwd=root, capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 1 and line["scaling"] == "weak" and line["value"] > 0
    assert line["parity"]["l1_ok"] and line["parity"]["l2_ok"], line["parity"]
    assert 0 < line["roofline"]["frac"] < 1
    assert line["local_probe_ms"] > 0 and line["partition_ms"] > 0 and line["exchange_ms"] >= 0
    assert line["xgmi_bytes_per_step"] == 0  # one rank: nothing crosses xGMI


@pytest.mark.parametrize("world,scaling", [(2, "weak"), (8, "weak"), (2, "strong"), (8, "strong")])
def test_bench_multi_rank_on_one_gpu(world, scaling):
    """The N > 1 HIP path as the driver's 8-GPU run takes it — bench.py --gpus N through its own
    launcher, N rank processes, DeviceOps with N owners (owner split into N destinations, the local
    table of 1/N of the build keys, received segments from N sources, the local partitioned probe) —
    with every rank on cuda:0 and gloo moving the all-to-alls through the host (RCCL refuses two
    ranks on one GPU; this box has one).  L1 + L2 of all ranks' probes exact, no fallback."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "2"
    p = subprocess.run([sys.executable, "bench.py", "--gpus", str(world), "--backend", "gloo", "--same-device",
                        "--steps", "2", "--warmup", "1", "--no-cpu", "--n-build-per-gpu", str(1 << 19),
                        "--n-probe", str(3 << 20), "--batches", "3", "--group", "2", "--scaling", scaling]
                       + (["--no-n1-same-shape"] if world == 8 else []),
                       cwd=root, capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and line["value"] > 0 and line["scaling"] == scaling
    assert line["config"]["n_probe_per_gpu"] == (3 << 20 if scaling == "weak" else (3 << 20) // world)
    assert line["parity"]["l1_ok"] and line["parity"]["l2_ok"], line["parity"]
    assert line["parity"]["exact_size_fallback_steps"] == 0
    assert line["xgmi_bytes_per_step"] > 0 and line["local_probe_ms"] > 0
    if world == 2:  # the curve's N = 1 point: the same per-GPU shape through the one-rank protocol
        ref = line["n1_same_shape"]
        assert line["n1_same_shape_ms"] == ref["ms_per_step"] > 0, ref
        assert ref["config"]["n_probe_per_gpu"] == line["config"]["n_probe_per_gpu"]
        assert ref["config"]["n_build_total"] == line["config"]["n_build_total"] // world
        assert line["per_gpu_value_vs_n1_same_shape"] > 0
