"""Multi-GPU radix-partitioned probe: one process per GPU, torch.distributed over
RCCL ("nccl" backend = RCCL on ROCm, xGMI between the GPUs of a node).

Per step, on every rank:
  1. owner partition of the local probe keys (ccj_partition_by_owner, HIP): destination-major keys
     + their global row ids, per-destination counts;
  2. all-to-all of the counts, then of keys and row ids (two all_to_all_single calls: the tuple
     shuffle over xGMI — the only data-path collective);
  3. local probe of the received keys against this rank's shard of the build side (ccj_probe);
  4. (verification only) all-reduce of match counts and of the order-insensitive L2 checksum.
The build side is sharded the same way once, before timing: every rank keeps the reference
generator's keys it owns and builds its local table on the device.

The exchange helpers are backend-agnostic, so tests/test_dist_cpu.py drives the same protocol with
the gloo backend on CPU tensors.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

import ccj


def exchange(send_keys, send_rows, send_counts, group=None):
    """All-to-all of destination-major (keys, rows) with per-destination counts (int64 tensor)."""
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc = [int(x) for x in send_counts.tolist()]
    rc = [int(x) for x in recv_counts.tolist()]
    n_send, n_recv = sum(sc), sum(rc)
    recv_keys = torch.empty(n_recv, dtype=send_keys.dtype, device=send_keys.device)
    recv_rows = torch.empty(n_recv, dtype=send_rows.dtype, device=send_rows.device)
    dist.all_to_all_single(recv_keys, send_keys[:n_send], rc, sc, group=group)
    dist.all_to_all_single(recv_rows, send_rows[:n_send], rc, sc, group=group)
    return recv_keys, recv_rows, rc


class ShardedProbe:
    """One rank's part of the multi-GPU probe of the C4 configuration."""

    def __init__(self, n_build_total: int, cf: int, n_probe: int, chunk: int, world: int, rank: int,
                 stream=None):
        self.world, self.rank, self.chunk, self.n_probe = world, rank, chunk, n_probe
        self.stream = stream
        dev = torch.device("cuda", torch.cuda.current_device())
        # build side: reference generator keys (linear_probing_ht.cpp:14-25) of the whole table,
        # generated in slices, each slice split by owner; this rank keeps its own part.
        own = []
        step = 1 << 26
        for b in range(0, n_build_total, step):
            n = min(step, n_build_total - b)
            keys = ccj.gen_reference_keys(b, n, n_build_total, cf, stream=stream)
            part = ccj.OwnerPartitioner(n, world, device=dev)
            k, _, cnt = part(keys, 0, stream=stream)
            torch.cuda.synchronize()
            c = cnt.tolist()
            lo = sum(c[:rank])
            own.append(k[lo:lo + c[rank]].clone())
        own_keys = torch.cat(own) if own else torch.empty(0, dtype=torch.int64, device=dev)
        self.n_build_local = own_keys.numel()
        self.table = ccj.Table.on_device(ccj.LP, own_keys, stream=stream)
        del own_keys
        self.part = ccj.OwnerPartitioner(n_probe, world, device=dev)
        self.out = None
        self.recv_rows = None

    def step(self, keys, row_base: int):
        k, r, cnt = self.part(keys, row_base, stream=self.stream)
        cur = torch.cuda.current_stream()
        if self.stream is not None:
            cur.wait_stream(self.stream)  # RCCL runs behind the current stream
        recv_keys, recv_rows, rc = exchange(k, r, cnt)
        if self.stream is not None:
            self.stream.wait_stream(cur)  # the probe runs behind the exchange
        n = recv_keys.numel()
        if self.out is None or self.out["n_chunks"] < (n + self.chunk - 1) // self.chunk:
            cap_rows = int(n * 1.05) + self.chunk
            self.out = self.table.alloc_outputs(cap_rows, self.chunk, rounds=True)
        out = dict(self.out)
        out["n_chunks"] = (n + self.chunk - 1) // self.chunk
        self.table.probe(recv_keys, self.chunk, out=out, stream=self.stream)
        self.recv_rows = recv_rows
        self.last = out
        return out, recv_keys, recv_rows
