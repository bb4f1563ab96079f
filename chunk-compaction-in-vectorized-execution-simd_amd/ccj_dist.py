"""Multi-GPU radix-partitioned probe: one process per GPU, torch.distributed over
RCCL ("nccl" backend = RCCL on ROCm, xGMI between the GPUs of a node).

Per step, on every rank, the 2^30 local probe keys go through in B batches, pipelined on three
HIP streams (partition, comm, probe) with double-buffered send/receive slots:
  1. owner partition of batch i (ccj_partition_by_owner_fixed, HIP): destination d's keys and u32
     row ids in fixed-capacity segment d, true counts beside them;
  2. all-to-all of counts and keys to the N - 1 peers with equal splits (all_to_all_single calls on
     the comm stream: the tuple shuffle over xGMI, the only data-path collective; no host round
     trip); the rank's own segment — last in its send buffer — is copied locally, never through
     RCCL (exchange_peers);
  3. local probe of the received segments, GROUP batches at a time (ccj_segment_chunk_counts +
     ccj_probe_partitioned: the live rows split by home-slot window, then walked with the window
     L2-resident) while the comm stream moves the next group's batches;
  4. (verification only) all-reduce of match counts and of the order-insensitive L2 checksum.
8 bytes cross xGMI per tuple in a timed step: the source rank is implied by the receive segment and
the source row by the position in it — the sender's owner split keeps every position's row in a row
buffer of that BATCH (one per batch of the step, kept until the batch is partitioned again in the
next step, i.e. longer than the receiver keeps the batch's probe results: two receive groups), so a
match (receive position, payload) names its probe tuple without the row travelling.  The rows can be
fetched afterwards (resolve_kept_groups: an untimed all-to-all of the kept row buffers); verify=True
moves them inside the step (a third all-to-all): its checksum needs global rows on the receiver.

Overflow.  Three things can overflow under key skew, each raising a flag in the rank's status
word: a send segment of the owner split, a receive segment's count, and the local probe's own
one-pass slot split or output capacity (its args->status IS the same word).  At the end of a run
(one or more steps issued back to back, ShardedProbe.run) the word is all-reduced with MAX, so
every rank sees the same value and takes the same branch: either all return, or all redo the run's
steps with the exact-size protocol (exchange(): host-side split sizes, 16 B per tuple) — the
ranks' collective sequences never diverge.

The step's control flow is written against an `ops` object: DeviceOps (below) runs the HIP kernels
on torch.cuda streams; tests/test_dist_cpu.py drives the SAME ShardedProbe with gloo on CPU
tensors and an oracle-backed ops object (batching, receive-group slots, group_row_map, the
overflow fallback on one rank only).
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.distributed as dist


# Largest buffer one all_to_all_single moves.  The RCCL in this image's torch wheel (2.26.6)
# corrupts a one-rank all_to_all_single from 1 GiB up (the first wrong element sits just past
# 512 MiB), so every exchange here is cut into batches of at most this size.
MAX_A2A_BYTES = 384 << 20
# Received batches probed together (one partitioned probe per group; each local probe sweeps the
# whole local table once).  One-rank rehearsal, step time with groups of 8 / 16 / 32
# batches: 37.4 / 36.0 / 34.8 ms; 16 keeps a probe overlapping the next group's exchange at N > 1.
GROUP = 16


def seg_capacity(n: int, world: int, chunk: int) -> int:
    """Receive-segment capacity for n keys hashed to `world` owners: the mean + 8 standard
    deviations + one chunk, rounded up to a multiple of chunk (probe chunks never straddle)."""
    mean = n / world
    cap = int(mean + 8 * math.sqrt(mean) + chunk)
    return (cap + chunk - 1) // chunk * chunk


def batch_count(n_probe: int, world: int, chunk: int, at_least: int = 1, subs: int = 1, cap=None) -> int:
    """Batches per step so that one batch's key buffer (world * subs segments of int64) fits
    MAX_A2A_BYTES.  cap(n): the sub-segment capacity for a batch of n keys."""
    cap = cap or (lambda n: seg_capacity(n, world * subs, chunk))
    b = max(1, at_least)
    while world * subs * cap(-(-n_probe // b)) * 8 > MAX_A2A_BYTES and b < n_probe:
        b *= 2
    return b


def slot_of(d: int, rank: int, world: int) -> int:
    """Slot of destination d in a rank's send buffers (ccj.h ccj_partition_by_owner_grouped,
    self_last = rank): the peers in rank order, then the rank's own region last."""
    return world - 1 if d == rank else d - (d > rank)


def exchange_peers(send, recv, per, world, rank, copy, group=None):
    """Move one buffer laid out in `world` slots of `per` elements (slots 0 .. world-2: the peers in
    rank order, slot world-1: the rank's own): ONE all_to_all_single with equal splits to the peers
    and a zero self split, so the peer regions are contiguous in rank order on both sides and no
    sizes travel through the host; the own slot never enters RCCL — `copy` moves it locally (at
    N = 8 an eighth of the bytes, which RCCL's copy kernel moved at ~0.75 TB/s)."""
    n = (world - 1) * per
    if world > 1:
        splits = [0 if d == rank else per for d in range(world)]
        dist.all_to_all_single(recv[:n], send[:n], splits, splits, group=group)
    copy(recv[n:n + per], send[n:n + per])


def exchange_fixed(send_keys, send_rows, send_counts, recv_keys, recv_rows, recv_counts, world, rank, seg, subs,
                   copy, group=None, rows=True):
    """All-to-all of fixed-capacity segments (slot layout of exchange_peers): seg keys (and rows)
    and subs counts per source.  rows=False: counts and keys only (a timed step: the rows stay
    with their sender)."""
    assert send_keys.numel() * send_keys.element_size() <= MAX_A2A_BYTES
    exchange_peers(send_counts, recv_counts, subs, world, rank, copy, group)
    exchange_peers(send_keys, recv_keys, seg, world, rank, copy, group)
    if rows:
        exchange_peers(send_rows, recv_rows, seg, world, rank, copy, group)


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


def agree_status(status, group=None) -> int:
    """MAX of every rank's status word: the one value all ranks branch on."""
    st = status.to(torch.int64) if status.dtype != torch.int64 else status.clone()
    dist.all_reduce(st, op=dist.ReduceOp.MAX, group=group)
    return int(st.item())


# CU split of the pipelined step, in groups of 8 CUs out of 32 (ccj.cu_mask_groups): the local
# probe's stream, the owner split's stream; the groups in neither stay free for RCCL's kernels.
# Without masks a local probe of ~3 * 10^5 workgroups holds every CU until it drains, and the owner
# split (one 149 KB-LDS workgroup per CU) and RCCL's kernels wait for it: no overlap at all
# (round-3 kernel trace of the one-rank rehearsal).  (0, 0): unmasked streams — the
# default until a split measures faster (one-rank rehearsal: 31.4 ms unmasked, 48.7 at (24, 8)).
CU_SPLIT = (0, 0)


class DeviceOps:
    """The HIP kernels (libccj.so) and torch.cuda streams/events one rank's step runs on."""

    def __init__(self, cu_split=None, share=True):
        """share: the local probe's split on 3/4 of the CUs (CCJ_PART_SHARE), leaving the rest to
        the exchange's RCCL kernels and the next owner splits."""
        import ccj
        self.ccj = ccj
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.cu_split = tuple(CU_SPLIT if cu_split is None else cu_split)
        self.share = share

    # streams and events
    def stream(self, role=None):
        """A stream for `role` ("probe", "partition"; None: any CUs)."""
        probe_g, part_g = self.cu_split
        if role and probe_g + part_g > 0:
            groups = range(probe_g) if role == "probe" else range(probe_g, probe_g + part_g)
            if role in ("probe", "partition") and len(groups):
                return self.ccj.cu_masked_stream(self.ccj.cu_mask_groups(set(groups)))
        return torch.cuda.Stream(device=self.device)

    def event(self, timing=False):
        return torch.cuda.Event(enable_timing=timing)

    def current(self):
        return torch.cuda.current_stream()

    def on(self, stream):
        return torch.cuda.stream(stream)

    def synchronize(self):
        torch.cuda.synchronize()

    # buffers
    def zeros(self, n, dtype):
        return torch.zeros(n, dtype=dtype, device=self.device)

    # build side: this rank's part of the reference generator's keys, built into a local LP table
    def build_local(self, n_build_total, cf, world, rank, stream):
        ccj = self.ccj
        own = []
        step = 1 << 26
        for b in range(0, n_build_total, step):
            n = min(step, n_build_total - b)
            keys = ccj.gen_reference_keys(b, n, n_build_total, cf, stream=stream)
            part = ccj.OwnerPartitioner(n, world, device=self.device)
            k, _, cnt = part(keys, 0, stream=stream)
            torch.cuda.synchronize()
            c = cnt.tolist()
            lo = sum(c[:rank])
            own.append(k[lo:lo + c[rank]].clone())
        own_keys = torch.cat(own) if own else torch.empty(0, dtype=torch.int64, device=self.device)
        self.table = ccj.Table.on_device(ccj.LP, own_keys, stream=stream)
        return own_keys.numel()

    # pipelined protocol
    # sub-segments per destination: the one-pass grouped partition fills one per XCD
    subs = 8

    def sub_capacity(self, n, world, chunk):
        return self.ccj.grouped_sub_cap(n, world, chunk)

    def fixed_partitioner(self, n, world, sub_cap, self_last):
        p = self.ccj.GroupedOwnerPartitioner(n, world, sub_cap, device=self.device, self_last=self_last)
        return lambda keys, row_base, sk, sr, sc, status, stream: p(keys, row_base, sk, sr, sc, status, stream=stream)

    def copy(self, dst, src):
        """dst[:] = src on the current stream (the rank's own segment: ccj_copy_device, 16-byte
        non-temporal loads and stores)."""
        if src.numel() * src.element_size() % 16 == 0:
            self.ccj.copy_device(dst, src, stream=torch.cuda.current_stream())
        else:
            dst.copy_(src)

    def segment_chunk_counts(self, seg_counts, seg_cap, chunk, out, status, stream):
        self.ccj.segment_chunk_counts(seg_counts, seg_cap, chunk, out, status, stream=stream)

    def alloc_group(self, gslots, chunk, status):
        """Partition workspace + outputs of one receive group; the probe reports into `status`."""
        part = self.table.alloc_partitioned(gslots, chunk)
        out = self.table.alloc_outputs(part["positions"], chunk, rounds=False)
        out["status"] = status
        return part, out

    def probe_group(self, keys, counts, part, out, chunk, stream):
        # share: the local split leaves CUs to RCCL and the next owner splits (ccj.h CCJ_PART_SHARE);
        # rows (CCJ_PART_ROWS, distinct build keys): the split writes every position's receive slot
        # and key into the outputs, so the walk writes only the chunks with a miss
        rows = int(self.table.max_dup) <= 1 and out["cap"] == chunk
        part["rows_mode"] = rows
        self.table.probe_partitioned(keys, chunk, counts=counts, out=out, part=part, stream=stream, retry=False,
                                     share=self.share, rows=rows)

    def group_rows(self, part, recv_rows, n_probe, seg_cap, slots, stream, src):
        """Global probe row of every position of a group's partitioned layout (gap positions hold
        arbitrary values: only matched positions are ever looked up); src[s] = the source rank of
        receive slot s."""
        n = recv_rows.numel()
        with torch.cuda.stream(stream):
            q = torch.arange(n, device=recv_rows.device) % slots
            srcs = torch.tensor(src, dtype=torch.int64, device=recv_rows.device)
            recv = srcs[q // seg_cap] * n_probe + recv_rows.to(torch.int64)
            if part.get("rows_mode"):  # out_sel holds receive slots: the map is by slot
                return recv
            rm = part["row_map"].to(torch.int64).clamp_(0, n - 1)
            return recv[rm]

    def checksum(self, out, chunk, row_map, stream):
        # rows mode: sel is the receive slot itself, so the map is read at sel (chunk 0)
        return self.ccj.result_checksum(out, 0 if out.get("rows_in_sel") else chunk, row_map=row_map, stream=stream)

    # exact-size protocol
    def owner_partitioner(self, n, world):
        p = self.ccj.OwnerPartitioner(n, world, device=self.device)
        return lambda keys, row_base, stream: p(keys, row_base, stream=stream)

    def probe_exact(self, keys, chunk, stream):
        return self.table.probe(keys, chunk, stream=stream, rounds=False)

    def probe_cost(self, keys, stream):
        return self.table.probe_cost(keys, stream=stream)


class ShardedProbe:
    """One rank's part of the multi-GPU probe of the C4 configuration."""

    def __init__(self, n_build_total: int, cf: int, n_probe: int, chunk: int, world: int, rank: int,
                 stream=None, batches: int = 4, ops=None, group=GROUP, keep_rows: bool = False):
        """keep_rows: one send-row buffer per batch (4 B per send slot and batch: 4.3 GB per rank
        at C4) instead of one per send slot, so that resolve_kept_groups can fetch a timed run's
        probe rows afterwards."""
        self.ops = ops or DeviceOps()
        self.keep_rows = keep_rows
        o = self.ops
        self.world, self.rank, self.chunk, self.n_probe = world, rank, chunk, n_probe
        # receive slot s holds source src_of_slot[s]'s segment (exchange_peers: peers, then own)
        self.src_of_slot = [0] * world
        for d in range(world):
            self.src_of_slot[slot_of(d, rank, world)] = d
        self.stream = stream or o.stream("probe")
        self.comm = o.stream()
        self.pstream = o.stream("partition")  # partitions run beside the previous probe
        self.n_build_local = o.build_local(n_build_total, cf, world, rank, self.stream)
        # batched, fixed-capacity exchange buffers: two send slots; receive buffers of `group`
        # batches each, two of them, so one group is probed while the next one arrives
        # a destination's region: `subs` sub-segments (the device partitioner fills one per XCD)
        self.subs = getattr(o, "subs", 1)
        sub_cap = getattr(o, "sub_capacity", None)
        cap = (lambda n: sub_cap(n, world, chunk)) if sub_cap else (lambda n: seg_capacity(n, world * self.subs, chunk))
        self.batches = batch_count(n_probe, world, chunk, batches, self.subs, cap)
        self.bn = -(-n_probe // self.batches)
        self.group = min(self.batches, group)
        self.n_groups = -(-self.batches // self.group)
        # the rank's status word: owner-split overflow, receive-count overflow and the local
        # probe's own flags (slot-split overflow, output capacity) all land here
        self.status = o.zeros(1, torch.int32)
        self._resize(cap(self.bn))
        ev = lambda: [o.event() for _ in range(2)]  # noqa: E731
        self.ev_part, self.ev_comm, self.ev_probe = ev(), ev(), ev()
        self.probe_events, self.part_events, self.comm_events = [], [], []
        self.parts_exact = {}  # exact-size partitioners (fallback), by batch size
        self.last_exact = False
        self.exact_steps = 0  # steps redone with the exact-size protocol (on every rank alike)

    def _resize(self, sub_cap: int):
        """(Re)allocate the exchange buffers for receive sub-segments of sub_cap slots (a source's
        region: subs of them, seg_cap slots)."""
        assert sub_cap % self.chunk == 0
        o = self.ops
        self.sub_cap = sub_cap
        self.seg_cap = seg_cap = self.subs * sub_cap
        self.nseg = self.world * self.subs  # received sub-segments per batch
        slots = self.world * seg_cap  # one batch's receive segments
        self.slots = slots
        gslots = self.group * slots
        self.fparts = {}
        mk = lambda dt, n: [o.zeros(n, dt) for _ in range(2)]  # noqa: E731
        self.sk, self.sc = mk(torch.int64, slots), mk(torch.int64, self.nseg)
        # send rows: with keep_rows one buffer per batch, so a timed step's matches stay traceable to
        # their probe rows after the step; otherwise one per send slot
        self.srb = [o.zeros(slots, torch.int32) for _ in range(self.batches if self.keep_rows else 2)]
        self.rk, self.rr = mk(torch.int64, gslots), mk(torch.int32, gslots)
        self.rc = mk(torch.int64, self.group * self.nseg)
        self.cc = mk(torch.int32, gslots // self.chunk)
        # local probe on the slot-partitioned path, one call per group of received batches
        self.parts, self.outs = [], []
        for _ in range(2):
            part, out = o.alloc_group(gslots, self.chunk, self.status)
            self.parts.append(part)
            self.outs.append(out)

    def _srb(self, j):
        """Send-row buffer of run batch j (per batch with keep_rows, else per send slot j % 2)."""
        return self.srb[j % self.batches] if self.keep_rows else self.srb[j % 2]

    def _batch(self, i):
        lo = i * self.bn
        return lo, min(self.bn, self.n_probe - lo)

    def _gslot(self, j):
        """Receive group slot of run batch j (batch j % batches of step j // batches): the groups of a
        run alternate between the two slots, across step boundaries too."""
        return ((j // self.batches) * self.n_groups + (j % self.batches) // self.group) % 2

    def _recv(self, j):
        """Receive views of run batch j: (group slot, keys, rows, counts)."""
        gs, sub = self._gslot(j), (j % self.batches) % self.group
        lo = sub * self.slots
        return (gs, self.rk[gs][lo:lo + self.slots], self.rr[gs][lo:lo + self.slots],
                self.rc[gs][sub * self.nseg:(sub + 1) * self.nseg])

    # ---- pipelined fixed-capacity step ----
    # Send slot s = i % 2 serves batches i, i+2, ...; receive group slot g % 2 serves groups g, g+2;
    # each reuse waits on the event of the previous user (events of the previous step included:
    # waiting on an unrecorded event is a no-op).
    def _timed(self, events, stream, timing):
        """Events around one piece of work on `stream` (timing steps only): its busy time."""
        if not timing:
            return contextlib.nullcontext()
        a, b = self.ops.event(True), self.ops.event(True)

        @contextlib.contextmanager
        def span():
            a.record(stream)
            yield
            b.record(stream)
            events.append((a, b))
        return span()

    def _partition(self, keys, j, timing=False):
        s = j % 2
        lo, n = self._batch(j % self.batches)
        if n not in self.fparts:
            self.fparts[n] = self.ops.fixed_partitioner(n, self.world, self.sub_cap, self.rank)
        self.pstream.wait_event(self.ev_comm[s])  # the previous all-to-all from send slot s is done
        with self._timed(self.part_events, self.pstream, timing):
            self.fparts[n](keys[lo:lo + n], lo, self.sk[s], self._srb(j), self.sc[s], self.status,
                           self.pstream)
        self.ev_part[s].record(self.pstream)

    def _exchange(self, j, timing=False, rows=True):
        s = j % 2
        gs, rk, rr, rc = self._recv(j)
        self.comm.wait_event(self.ev_part[s])
        if (j % self.batches) % self.group == 0:
            self.comm.wait_event(self.ev_probe[gs])  # the previous probe of receive group slot gs is done
        with self.ops.on(self.comm), self._timed(self.comm_events, self.comm, timing):
            exchange_fixed(self.sk[s], self._srb(j), self.sc[s], rk, rr, rc, self.world, self.rank,
                           self.seg_cap, self.subs, self.ops.copy, rows=rows)
        self.ev_comm[s].record(self.comm)

    def reset_timing(self):
        self.probe_events.clear()
        self.part_events.clear()
        self.comm_events.clear()

    def timing_ms(self, steps: int) -> dict:
        """Per step (mean over the timed steps): busy time of the partition, exchange and local-probe
        streams.  The three overlap (pipelined), so they bound the step from below, not add up."""
        tot = lambda evs: sum(a.elapsed_time(b) for a, b in evs) / max(steps, 1)  # noqa: E731
        return {"partition_ms": tot(self.part_events), "exchange_ms": tot(self.comm_events),
                "local_probe_ms": tot(self.probe_events)}

    def xgmi_bytes_per_step(self) -> dict:
        """Bytes this rank sends to the other ranks per timed step: the fixed-capacity segments move
        whole (equal splits: keys 8 B per slot, one count per sub-segment; the rows stay with their
        sender), and the expected live part of them for uniform keys (8 B per tuple that changes
        GPU)."""
        peers = self.world - 1
        per_batch = peers * (self.seg_cap * 8 + self.subs * 8)
        return {"sent_to_peers": self.batches * per_batch,
                "useful_to_peers": self.n_probe * peers / self.world * 8}

    def _group_range(self, g):
        return g * self.group, min((g + 1) * self.group, self.batches) - 1

    def _probe(self, j0, g, timing):
        """Probe group g of the step whose first run batch is j0 (batches g*group ... its last one,
        all exchanged in order on comm)."""
        o = self.ops
        first, last = self._group_range(g)
        gs = self._gslot(j0 + first)
        self.stream.wait_event(self.ev_comm[(j0 + last) % 2])
        per = self.slots // self.chunk
        for i in range(first, last + 1):
            sub = i % self.group
            o.segment_chunk_counts(self.rc[gs][sub * self.nseg:(sub + 1) * self.nseg], self.sub_cap, self.chunk,
                                   self.cc[gs][sub * per:(sub + 1) * per], self.status, self.stream)
        if last - first + 1 < self.group:  # a short last group: its missing batches have no live rows
            with o.on(self.stream):
                self.cc[gs][(last - first + 1) * per:].zero_()
        if timing:
            a, b = o.event(True), o.event(True)
            a.record(self.stream)
        o.probe_group(self.rk[gs], self.cc[gs], self.parts[gs], self.outs[gs], self.chunk, self.stream)
        if timing:
            b.record(self.stream)
            self.probe_events.append((a, b))
        self.ev_probe[gs].record(self.stream)

    def group_row_map(self, j0, g):
        gs = self._gslot(j0 + self._group_range(g)[0])
        return self.ops.group_rows(self.parts[gs], self.rr[gs], self.n_probe, self.seg_cap, self.slots, self.stream,
                                   self.src_of_slot)

    def received_keys(self, i):
        """Batch i's received keys (of the last run's first step: call after a one-step run) without
        the segment padding (work accounting)."""
        gs, rk, rr, rc = self._recv(i)
        self.ops.current().wait_event(self.ev_comm[i % 2])
        pos = torch.arange(self.slots, device=rk.device)
        live = (pos % self.sub_cap) < rc[pos // self.sub_cap]
        return rk[live]

    def step(self, keys, row_base: int = 0, timing: bool = False, verify: bool = False):
        """One pass over this rank's keys.  verify=True returns (matches, l2) of this rank's probes
        (global rows: source rank * n_probe + local row)."""
        return self.run(keys, row_base, 1, timing, verify)

    def run(self, keys, row_base: int = 0, steps: int = 1, timing: bool = False, verify: bool = False):
        """`steps` passes over this rank's keys, issued back to back: the batches of step s + 1 are
        partitioned and exchanged while step s's last group is probed (no drain between steps), and
        the status word is agreed on once, after the last step.  If any rank saw an overflow, every
        rank redoes all `steps` passes with the exact-size protocol.  verify=True returns (matches,
        l2) summed over the steps."""
        o = self.ops
        assert keys.numel() == self.n_probe and row_base == self.rank * self.n_probe and steps >= 1
        cur = o.current()
        with o.on(cur):
            self.status.zero_()
        self.stream.wait_stream(cur)
        self.pstream.wait_stream(cur)
        total = steps * self.batches  # run batches j: batch j % batches of step j // batches
        self._run_steps = steps
        self._partition(keys, 0, timing)
        self._exchange(0, timing, rows=verify)
        m, l2 = 0, 0
        for j in range(total):
            if j + 1 < total:
                self._partition(keys, j + 1, timing)
                self._exchange(j + 1, timing, rows=verify)
            i, j0 = j % self.batches, j - j % self.batches
            if i % self.group == self.group - 1 or i == self.batches - 1:  # group i // group complete
                g = i // self.group
                self._probe(j0, g, timing)
                if verify:
                    gs = self._gslot(j)
                    bm, bl = o.checksum(self.outs[gs], self.chunk, self.group_row_map(j0, g), self.stream)
                    m, l2 = m + bm, (l2 + bl) % (1 << 64)
                    # the next user of receive slot gs waits for the verification's reads of it too
                    self.ev_probe[gs].record(self.stream)
        cur.wait_stream(self.stream)
        cur.wait_stream(self.pstream)
        cur.wait_stream(self.comm)
        # Every rank branches on the same value: the MAX of all ranks' status words.
        if agree_status(self.status):
            self.last_exact = True
            self.exact_steps += steps
            m, l2 = 0, 0
            for _ in range(steps):
                r = self.step_exact(keys, row_base, verify)
                if verify:
                    m, l2 = m + r[0], (l2 + r[1]) % (1 << 64)
            return (m, l2) if verify else None
        self.last_exact = False
        return (m, l2) if verify else None

    def resolve_kept_groups(self):
        """After a timed (key-only) run: fetch the probe rows of the groups whose results are still
        held (the run's last two groups — the receive slots alternate) from their senders' kept
        per-batch row buffers, with an untimed all-to-all per batch, and return (matches, l2 over
        global rows, batch indices covered).  Shows that a timed step's matches name their probe
        tuples although no row crossed during it.  Call right after run() (no verify)."""
        o = self.ops
        if not self.keep_rows:
            raise RuntimeError("resolve_kept_groups needs ShardedProbe(..., keep_rows=True)")
        if self.last_exact:
            raise RuntimeError("the last run fell back to the exact-size protocol: nothing kept")
        o.synchronize()
        groups = list(range(max(0, self.n_groups - 2), self.n_groups))
        j0 = (self._run_steps - 1) * self.batches  # the run's last step
        m, l2, covered = 0, 0, []
        for g in groups:
            first, last = self._group_range(g)
            for i in range(first, last + 1):
                gs, rk, rr, rc = self._recv(j0 + i)
                with o.on(self.comm):
                    exchange_peers(self.srb[i], rr, self.seg_cap, self.world, self.rank, o.copy)
                covered.append(i)
            self.stream.wait_stream(self.comm)
            gs = self._gslot(j0 + first)
            bm, bl = o.checksum(self.outs[gs], self.chunk, self.group_row_map(j0, g), self.stream)
            m, l2 = m + bm, (l2 + bl) % (1 << 64)
        o.synchronize()
        return m, l2, covered

    def probe_alone_ms(self, reps: int = 3, share=None) -> float:
        """After a run: the run's last group probed again with nothing else on the device (every
        stream drained first) — the local probe's own time, beside `local_probe_ms`, which is its
        busy time while the partition and exchange streams share the GPU.  Min over `reps`.
        share (DeviceOps only): override the ops' CU share for these probes (False: the whole grid,
        the kernels' own speed without the room the step leaves to the exchange and owner splits)."""
        o = self.ops
        if self.last_exact:
            raise RuntimeError("the last run fell back to the exact-size protocol")
        if share is not None and hasattr(o, "share"):
            saved = o.share
            o.share = share
            try:
                return self.probe_alone_ms(reps)
            finally:
                o.share = saved
        o.synchronize()
        g = self.n_groups - 1
        first, _ = self._group_range(g)
        gs = self._gslot((self._run_steps - 1) * self.batches + first)
        best = None
        for _ in range(reps):
            a, b = o.event(True), o.event(True)
            a.record(self.stream)
            o.probe_group(self.rk[gs], self.cc[gs], self.parts[gs], self.outs[gs], self.chunk, self.stream)
            b.record(self.stream)
            o.synchronize()
            t = a.elapsed_time(b)
            best = t if best is None else min(best, t)
        return best

    # ---- exact-size protocol (fallback for skewed keys), batch by batch, not overlapped ----
    def step_exact(self, keys, row_base: int, verify: bool = False):
        o = self.ops
        o.synchronize()
        m, l2 = 0, 0
        for i in range(self.batches):
            lo, n = self._batch(i)
            if n not in self.parts_exact:
                self.parts_exact[n] = o.owner_partitioner(n, self.world)
            k, r, cnt = self.parts_exact[n](keys[lo:lo + n], row_base + lo, self.stream)
            cur = o.current()
            cur.wait_stream(self.stream)  # RCCL runs behind the current stream
            recv_keys, recv_rows, rc = exchange(k, r, cnt)
            self.stream.wait_stream(cur)  # the probe runs behind the exchange
            out = o.probe_exact(recv_keys, self.chunk, self.stream)
            if verify:
                bm, bl = o.checksum(out, self.chunk, recv_rows, self.stream)
                m, l2 = m + bm, (l2 + bl) % (1 << 64)
            o.synchronize()
        return (m, l2) if verify else None


class HostStream:
    """Stand-in for a HIP stream on CPU tensors: work runs in program order, so ordering is trivial."""

    def wait_event(self, ev):
        pass

    def wait_stream(self, other):
        pass

    def synchronize(self):
        pass


class HostEvent:
    def record(self, stream=None):
        pass

    def elapsed_time(self, other):
        return 0.0


class HostOpsBase:
    """Stream/event/buffer half of a CPU ops object (tests/test_dist_cpu.py supplies the kernels'
    stand-ins on top of it)."""

    device = torch.device("cpu")

    def stream(self, role=None):
        return HostStream()

    def event(self, timing=False):
        return HostEvent()

    def current(self):
        return HostStream()

    def on(self, stream):
        return contextlib.nullcontext()

    def synchronize(self):
        pass

    def zeros(self, n, dtype):
        return torch.zeros(n, dtype=dtype)

    def copy(self, dst, src):
        dst.copy_(src)
