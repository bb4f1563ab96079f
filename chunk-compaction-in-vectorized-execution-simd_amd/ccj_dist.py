"""Multi-GPU radix-partitioned probe: one process per GPU, torch.distributed over
RCCL ("nccl" backend = RCCL on ROCm, xGMI between the GPUs of a node).

Per step, on every rank, the 2^30 local probe keys go through in B batches, pipelined on three
HIP streams (partition, comm, probe) with double-buffered send/receive slots:
  1. owner partition of batch i (ccj_partition_by_owner_fixed, HIP): destination d's keys and u32
     row ids in fixed-capacity segment d, true counts beside them;
  2. all-to-all of counts, keys, rows with equal splits (three all_to_all_single calls on the comm
     stream: the tuple shuffle over xGMI, the only data-path collective; no host round trip);
  3. local probe of the received segments, GROUP batches at a time (ccj_segment_chunk_counts +
     ccj_probe_partitioned: the live rows split by home-slot window, then walked with the window
     L2-resident) while the comm stream moves the next group's batches;
  4. (verification only) all-reduce of match counts and of the order-insensitive L2 checksum.
12 bytes cross xGMI per tuple (the source rank is implied by the receive segment).  A segment
that overflows its capacity (skewed keys) is detected on the device; that step is then redone
with the exact-size protocol (exchange(): host-side split sizes, 16 B per tuple).
The build side is sharded the same way once, before timing: every rank keeps the reference
generator's keys it owns and builds its local table on the device.

The exchange helpers are backend-agnostic, so tests/test_dist_cpu.py drives the same protocol with
the gloo backend on CPU tensors.
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist

import ccj


# Largest buffer one all_to_all_single moves.  The RCCL in this image's torch wheel (2.26.6)
# corrupts a one-rank all_to_all_single from 1 GiB up (tools/dbg_a2a.py: the first wrong element
# sits just past 512 MiB), so every exchange here is cut into batches of at most this size.
MAX_A2A_BYTES = 384 << 20
# Received batches probed together (one partitioned probe per group): 8 x 2^25 keys at C4.
# One-rank rehearsal, local probe per step: groups of 2 / 4 / 8 batches 30.6 / 25.6 / 23.9 ms.
GROUP = int(os.environ.get("CCJ_SHARD_GROUP", "8"))


def seg_capacity(n: int, world: int, chunk: int) -> int:
    """Receive-segment capacity for n keys hashed to `world` owners: the mean + 8 standard
    deviations + one chunk, rounded up to a multiple of chunk (probe chunks never straddle)."""
    mean = n / world
    cap = int(mean + 8 * math.sqrt(mean) + chunk)
    return (cap + chunk - 1) // chunk * chunk


def batch_count(n_probe: int, world: int, chunk: int, at_least: int = 1) -> int:
    """Batches per step so that one batch's key buffer (world segments of int64) fits MAX_A2A_BYTES."""
    b = max(1, at_least)
    while world * seg_capacity(-(-n_probe // b), world, chunk) * 8 > MAX_A2A_BYTES and b < n_probe:
        b *= 2
    return b


def exchange_fixed(send_keys, send_rows, send_counts, recv_keys, recv_rows, recv_counts, group=None):
    """All-to-all of fixed-capacity segments: equal splits, so no sizes travel through the host."""
    assert send_keys.numel() * send_keys.element_size() <= MAX_A2A_BYTES
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    dist.all_to_all_single(recv_keys, send_keys, group=group)
    dist.all_to_all_single(recv_rows, send_rows, group=group)


def exchange(send_keys, send_rows, send_counts, group=None):
    """All-to-all of destination-major (keys, rows) with per-destination counts (int64 tensor)."""
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc = [int(x) for x in send_counts.tolist()]
    rc = [int(x) for x in recv_counts.tolist()]
    n_send, n_recv = sum(sc), sum(rc)
    assert max(n_send, n_recv) * 8 <= MAX_A2A_BYTES, "exchange larger than one all_to_all may move"
    recv_keys = torch.empty(n_recv, dtype=send_keys.dtype, device=send_keys.device)
    recv_rows = torch.empty(n_recv, dtype=send_rows.dtype, device=send_rows.device)
    dist.all_to_all_single(recv_keys, send_keys[:n_send], rc, sc, group=group)
    dist.all_to_all_single(recv_rows, send_rows[:n_send], rc, sc, group=group)
    return recv_keys, recv_rows, rc


class ShardedProbe:
    """One rank's part of the multi-GPU probe of the C4 configuration."""

    def __init__(self, n_build_total: int, cf: int, n_probe: int, chunk: int, world: int, rank: int,
                 stream=None, batches: int = 4):
        self.world, self.rank, self.chunk, self.n_probe = world, rank, chunk, n_probe
        dev = torch.device("cuda", torch.cuda.current_device())
        self.stream = stream or torch.cuda.Stream(device=dev)
        self.comm = torch.cuda.Stream(device=dev)
        self.pstream = torch.cuda.Stream(device=dev)  # partitions run beside the previous probe
        # build side: reference generator keys (linear_probing_ht.cpp:14-25) of the whole table,
        # generated in slices, each slice split by owner; this rank keeps its own part.
        own = []
        step = 1 << 26
        for b in range(0, n_build_total, step):
            n = min(step, n_build_total - b)
            keys = ccj.gen_reference_keys(b, n, n_build_total, cf, stream=self.stream)
            part = ccj.OwnerPartitioner(n, world, device=dev)
            k, _, cnt = part(keys, 0, stream=self.stream)
            torch.cuda.synchronize()
            c = cnt.tolist()
            lo = sum(c[:rank])
            own.append(k[lo:lo + c[rank]].clone())
        own_keys = torch.cat(own) if own else torch.empty(0, dtype=torch.int64, device=dev)
        self.n_build_local = own_keys.numel()
        self.table = ccj.Table.on_device(ccj.LP, own_keys, stream=self.stream)
        del own_keys
        # batched, fixed-capacity exchange buffers: two send slots; receive buffers of `group`
        # batches each, two of them, so one group is probed while the next one arrives
        self.batches = batch_count(n_probe, world, chunk, batches)
        self.bn = -(-n_probe // self.batches)
        self.group = min(self.batches, GROUP)
        self.n_groups = -(-self.batches // self.group)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self._resize(seg_capacity(self.bn, world, chunk))
        ev = lambda: [torch.cuda.Event() for _ in range(2)]  # noqa: E731
        self.ev_part, self.ev_comm, self.ev_probe = ev(), ev(), ev()
        self.probe_events = []
        self.parts_exact = {}  # exact-size partitioners (fallback), by batch size
        self.last_exact = False

    def _resize(self, seg_cap: int):
        """(Re)allocate the exchange buffers for receive segments of seg_cap slots."""
        assert seg_cap % self.chunk == 0
        dev = torch.device("cuda", torch.cuda.current_device())
        self.seg_cap = seg_cap
        slots = self.world * seg_cap  # one batch's receive segments
        self.slots = slots
        gslots = self.group * slots
        self.fparts = {}
        mk = lambda dt, n: [torch.zeros(n, dtype=dt, device=dev) for _ in range(2)]  # noqa: E731
        self.sk, self.sr, self.sc = mk(torch.int64, slots), mk(torch.int32, slots), mk(torch.int64, self.world)
        self.rk, self.rr = mk(torch.int64, gslots), mk(torch.int32, gslots)
        self.rc = mk(torch.int64, self.group * self.world)
        self.cc = mk(torch.int32, gslots // self.chunk)
        # local probe on the slot-partitioned path, one call per group of received batches: the
        # live rows (per-chunk counts) are split by home-slot window, then walked with the table
        # window L2-resident; a group of batches makes segments long enough to fill chunks
        self.parts = [self.table.alloc_partitioned(gslots, self.chunk) for _ in range(2)]
        self.outs = [self.table.alloc_outputs(p["positions"], self.chunk, rounds=False) for p in self.parts]

    def _batch(self, i):
        lo = i * self.bn
        return lo, min(self.bn, self.n_probe - lo)

    def _recv(self, i):
        """Receive views of batch i: (group slot, keys, rows, counts)."""
        gs, sub = (i // self.group) % 2, i % self.group
        lo = sub * self.slots
        return (gs, self.rk[gs][lo:lo + self.slots], self.rr[gs][lo:lo + self.slots],
                self.rc[gs][sub * self.world:(sub + 1) * self.world])

    # ---- pipelined fixed-capacity step ----
    # Send slot s = i % 2 serves batches i, i+2, ...; receive group slot g % 2 serves groups g, g+2;
    # each reuse waits on the event of the previous user (events of the previous step included:
    # waiting on an unrecorded event is a no-op).
    def _partition(self, keys, i):
        s = i % 2
        lo, n = self._batch(i)
        if n not in self.fparts:
            self.fparts[n] = ccj.FixedOwnerPartitioner(n, self.world, self.seg_cap, device=keys.device)
        self.pstream.wait_event(self.ev_comm[s])  # the previous all-to-all from send slot s is done
        self.fparts[n](keys[lo:lo + n], lo, self.sk[s], self.sr[s], self.sc[s], self.status, stream=self.pstream)
        self.ev_part[s].record(self.pstream)

    def _exchange(self, i):
        s = i % 2
        gs, rk, rr, rc = self._recv(i)
        self.comm.wait_event(self.ev_part[s])
        if i % self.group == 0:
            self.comm.wait_event(self.ev_probe[gs])  # the previous probe of receive group slot gs is done
        with torch.cuda.stream(self.comm):
            exchange_fixed(self.sk[s], self.sr[s], self.sc[s], rk, rr, rc)
        self.ev_comm[s].record(self.comm)

    def _probe(self, g, timing):
        """Probe group g (batches g*group ... its last one, all exchanged in order on comm)."""
        gs = g % 2
        first, last = g * self.group, min((g + 1) * self.group, self.batches) - 1
        self.stream.wait_event(self.ev_comm[last % 2])
        per = self.slots // self.chunk
        for i in range(first, last + 1):
            sub = i % self.group
            ccj.segment_chunk_counts(self.rc[gs][sub * self.world:(sub + 1) * self.world], self.seg_cap, self.chunk,
                                     self.cc[gs][sub * per:(sub + 1) * per], self.status, stream=self.stream)
        if last - first + 1 < self.group:  # a short last group: its missing batches have no live rows
            with torch.cuda.stream(self.stream):
                self.cc[gs][(last - first + 1) * per:].zero_()
        if timing:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(self.stream)
        self.table.probe_partitioned(self.rk[gs], self.chunk, counts=self.cc[gs], out=self.outs[gs],
                                     part=self.parts[gs], stream=self.stream, retry=False)
        if timing:
            b.record(self.stream)
            self.probe_events.append((a, b))
        self.ev_probe[gs].record(self.stream)

    def group_row_map(self, g):
        """Global probe row of every position of group g's partitioned layout (gap positions hold
        arbitrary values: only matched positions are ever looked up)."""
        gs = g % 2
        n = self.group * self.slots
        with torch.cuda.stream(self.stream):  # behind this group's probe, before the slot's next use
            q = torch.arange(n, device=self.rr[gs].device) % self.slots
            recv = (q // self.seg_cap) * self.n_probe + self.rr[gs].to(torch.int64)
            rm = self.parts[gs]["row_map"].to(torch.int64).clamp_(0, n - 1)
            return recv[rm]

    def received_keys(self, i):
        """Batch i's received keys without the segment padding (work accounting)."""
        gs, rk, rr, rc = self._recv(i)
        torch.cuda.current_stream().wait_event(self.ev_comm[i % 2])
        pos = torch.arange(self.slots, device=rk.device)
        live = (pos % self.seg_cap) < rc[pos // self.seg_cap]
        return rk[live]

    def step(self, keys, row_base: int = 0, timing: bool = False, verify: bool = False):
        """One pass over this rank's keys.  verify=True returns (matches, l2) of this rank's probes
        (global rows: source rank * n_probe + local row)."""
        assert keys.numel() == self.n_probe and row_base == self.rank * self.n_probe
        self.status.zero_()
        self.stream.wait_stream(torch.cuda.current_stream())
        self.pstream.wait_stream(torch.cuda.current_stream())
        self._partition(keys, 0)
        self._exchange(0)
        m, l2 = 0, 0
        for i in range(self.batches):
            if i + 1 < self.batches:
                self._partition(keys, i + 1)
                self._exchange(i + 1)
            if i % self.group == self.group - 1 or i == self.batches - 1:  # group i // group complete
                g = i // self.group
                self._probe(g, timing)
                if verify:
                    bm, bl = ccj.result_checksum(self.outs[g % 2], self.chunk, row_map=self.group_row_map(g),
                                                 stream=self.stream)
                    m, l2 = m + bm, (l2 + bl) % (1 << 64)
        torch.cuda.current_stream().wait_stream(self.stream)
        torch.cuda.current_stream().wait_stream(self.pstream)
        if int(self.status.item()):  # a fixed-capacity segment overflowed: redo with exact sizes
            self.last_exact = True
            return self.step_exact(keys, row_base, verify)
        self.last_exact = False
        return (m, l2) if verify else None

    # ---- exact-size protocol (fallback for skewed keys), batch by batch, not overlapped ----
    def step_exact(self, keys, row_base: int, verify: bool = False):
        torch.cuda.synchronize()
        m, l2 = 0, 0
        for i in range(self.batches):
            lo, n = self._batch(i)
            if n not in self.parts_exact:
                self.parts_exact[n] = ccj.OwnerPartitioner(n, self.world, device=keys.device)
            k, r, cnt = self.parts_exact[n](keys[lo:lo + n], row_base + lo, stream=self.stream)
            cur = torch.cuda.current_stream()
            cur.wait_stream(self.stream)  # RCCL runs behind the current stream
            recv_keys, recv_rows, rc = exchange(k, r, cnt)
            self.stream.wait_stream(cur)  # the probe runs behind the exchange
            out = self.table.probe(recv_keys, self.chunk, stream=self.stream, rounds=False)
            if verify:
                bm, bl = ccj.result_checksum(out, self.chunk, row_map=recv_rows, stream=self.stream)
                m, l2 = m + bm, (l2 + bl) % (1 << 64)
            torch.cuda.synchronize()
        return (m, l2) if verify else None
