"""Python binding of libccj.so (include/ccj.h) over ctypes.

PyTorch is plumbing here: device buffers are torch tensors on `cuda:N` and streams are torch
streams; every computation runs in the HIP kernels of libccj.so.  There is no CPU fallback —
loading fails loudly when the library is missing, and every call fails without a gfx950 device.

Mirrors the reference operator surface for the probe path:
  Table.reference(kind, n, cf)   <- LPHashTable(n, cf) / HashTable(n, cf)  (linear_probing_ht.cpp:4-37,
                                    chaining_ht.cpp:4-36)
  Table.probe(keys, chunk, ...)  <- Probe + `while HasNext(): Next(...)`    (linear_probing_ht.cpp:39-115,
                                    chaining_ht.cpp:38-136), batched over chunks
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
# the product library; CCJ_LIB_PATH names another build (tests/test_rank_gpu.py runs the rank walk's
# checks against libccj_tuning.so, the only build that contains it)
LIB_PATH = os.environ.get("CCJ_LIB_PATH") or os.path.join(HERE, "libccj.so")

LP, CHAIN = 0, 1
LAYOUT_REFERENCE, LAYOUT_DEVICE = 0, 1
FLAG_CAP_OVERFLOW, FLAG_ROUND_OVERFLOW, FLAG_BAD_INPUT, FLAG_PART_OVERFLOW = 1, 2, 4, 8
PART_EXACT = 1
PART_ROWS = 2  # out_sel = the original row of every match (ccj.h CCJ_PART_ROWS)
PART_RANK = 4  # the rank walk (LDS window index; libccj_tuning.so only) instead of the slot-array walk
PART_SHARE = 8  # the split leaves 1/4 of the CUs to other streams (ccj.h CCJ_PART_SHARE; multi-GPU step)

_lib = None
ABI_VERSION = 15  # include/ccj.h CCJ_ABI_VERSION this binding is written against


class CCJError(RuntimeError):
    pass


class TableInfo(C.Structure):
    _fields_ = [("kind", C.c_int32), ("layout", C.c_int32), ("n_keys", C.c_uint64), ("size", C.c_uint64),
                ("max_dup", C.c_uint64), ("max_rounds", C.c_uint32), ("reserved", C.c_uint32),
                ("d_table", C.c_void_p), ("d_bucket_off", C.c_void_p)]


class TableArrays(C.Structure):
    _fields_ = [("d_table", C.c_void_p), ("positions", C.c_uint64), ("d_row", C.c_void_p),
                ("d_bucket_off", C.c_void_p), ("d_bucket16", C.c_void_p), ("d_bucket8", C.c_void_p),
                ("n_bucket8", C.c_uint64), ("d_bucket_filter", C.c_void_p), ("n_filter_words", C.c_uint64)]


class ProbeArgs(C.Structure):
    _fields_ = [("keys", C.c_void_p), ("sel", C.c_void_p), ("counts", C.c_void_p), ("n_rows", C.c_uint64),
                ("chunk", C.c_uint32), ("max_rounds", C.c_uint32), ("cap", C.c_uint64),
                ("out_count", C.c_void_p), ("out_sel", C.c_void_p), ("out_payload", C.c_void_p),
                ("out_rounds", C.c_void_p), ("out_round_counts", C.c_void_p), ("status", C.c_void_p),
                ("out_pos", C.c_void_p), ("n_payload_cols", C.c_uint32), ("reserved2", C.c_uint32),
                ("out_payload_cols", C.c_void_p * 8)]


class CompactArgs(C.Structure):
    _fields_ = [("count", C.c_void_p), ("sel", C.c_void_p), ("payload", C.c_void_p), ("rounds", C.c_void_p),
                ("round_counts", C.c_void_p), ("n_chunks", C.c_uint64), ("cap", C.c_uint64),
                ("max_rounds", C.c_uint32), ("chunk", C.c_uint32), ("n_cols", C.c_uint32), ("threshold", C.c_uint32),
                ("cols", C.c_void_p * 16), ("out_cols", C.c_void_p * 16), ("out_payload", C.c_void_p),
                ("out_row", C.c_void_p), ("out_chunk_counts", C.c_void_p), ("out_cap_rows", C.c_uint64),
                ("out_n_chunks", C.c_void_p), ("workspace", C.c_void_p), ("workspace_bytes", C.c_size_t),
                ("status", C.c_void_p), ("key_cols", C.c_uint32)]


EXPORTS = ["ccj_last_error", "ccj_abi_version", "ccj_device_init", "ccj_table_build_reference",
           "ccj_table_build_from_host", "ccj_table_build_on_device", "ccj_table_get_info", "ccj_table_free",
           "ccj_probe", "ccj_gen_uniform_keys", "ccj_probe_cost", "ccj_result_checksum",
           "ccj_compact_workspace_size", "ccj_compact", "ccj_partition_workspace_size", "ccj_partition_by_owner",
           "ccj_result_checksum_mapped", "ccj_gen_reference_keys", "ccj_table_set_payload",
           "ccj_table_build_rank_index",
           "ccj_probe_partitioned_workspace_size", "ccj_probe_partitioned", "ccj_probe_partitioned_positions",
           "ccj_pipeline_create",
           "ccj_pipeline_run", "ccj_pipeline_free", "ccj_pipeline_checksum", "ccj_partition_by_owner_fixed",
           "ccj_segment_chunk_counts", "ccj_pipeline_set_thresholds", "ccj_gen_c3_keys",
           "ccj_partition_grouped_workspace_size", "ccj_partition_by_owner_grouped", "ccj_partition_grouped_sub_cap",
           "ccj_probe_ordered_workspace_size", "ccj_probe_ordered", "ccj_probe_visits",
           "ccj_stream_create_cu_masked", "ccj_stream_destroy", "ccj_device_cus", "ccj_copy_device",
           "ccj_table_get_arrays", "ccj_probe_cost_walk", "ccj_set_phase_events", "ccj_build_hash",
           "ccj_last_gather_kernel"]

MAX_JOINS = 8
COMPACT_NONE, COMPACT_FULL = 0, 1


class PipelineResult(C.Structure):
    _fields_ = [("n_out", C.c_uint64), ("cols", C.c_void_p * MAX_JOINS), ("payload", C.c_void_p * MAX_JOINS),
                ("chunks_in", C.c_uint64 * MAX_JOINS), ("rows_in", C.c_uint64 * MAX_JOINS),
                ("rows_out", C.c_uint64 * MAX_JOINS), ("level_ms", C.c_float * MAX_JOINS)]


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "-j8"], check=True)
    return LIB_PATH


def lib():
    """Load libccj.so (in-tree).  Raises if it is missing: there is no fallback path."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CCJError(f"{LIB_PATH} missing: run `make -C {HERE}` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp, u64, i32 = C.c_void_p, C.c_uint64, C.c_int
        L.ccj_last_error.restype = C.c_char_p
        L.ccj_abi_version.restype = i32
        if L.ccj_abi_version() != ABI_VERSION:  # a stale build would shift every later argument
            raise CCJError(f"{LIB_PATH} has ABI {L.ccj_abi_version()}, this binding needs {ABI_VERSION}: "
                           f"rebuild it (`make -C {HERE}`)")
        L.ccj_build_hash.restype = C.c_char_p
        L.ccj_last_gather_kernel.restype = C.c_char_p
        L.ccj_device_init.argtypes = [i32]
        L.ccj_table_build_reference.argtypes = [i32, u64, u64, i32, vp, C.POINTER(vp)]
        L.ccj_table_build_from_host.argtypes = [i32, vp, u64, C.POINTER(vp)]
        L.ccj_table_build_on_device.argtypes = [i32, vp, u64, vp, C.POINTER(vp)]
        L.ccj_table_get_info.argtypes = [vp, C.POINTER(TableInfo)]
        L.ccj_table_get_arrays.argtypes = [vp, C.POINTER(TableArrays)]
        L.ccj_table_free.argtypes = [vp]
        L.ccj_table_set_payload.argtypes = [vp, vp, C.c_uint32, vp]
        L.ccj_table_build_rank_index.argtypes = [vp, vp]
        L.ccj_probe_partitioned_workspace_size.restype = C.c_size_t
        L.ccj_probe_partitioned_workspace_size.argtypes = [vp, u64, C.c_uint32]
        L.ccj_probe_partitioned_positions.restype = u64
        L.ccj_probe_partitioned_positions.argtypes = [vp, u64, C.c_uint32]
        L.ccj_probe_partitioned.argtypes = [vp, C.POINTER(ProbeArgs), C.c_uint32, vp, vp, C.c_size_t, vp]
        L.ccj_probe.argtypes = [vp, C.POINTER(ProbeArgs), vp]
        L.ccj_probe_ordered_workspace_size.restype = C.c_size_t
        L.ccj_probe_ordered_workspace_size.argtypes = [vp, u64, C.c_uint32]
        L.ccj_probe_ordered.argtypes = [vp, C.POINTER(ProbeArgs), vp, C.c_size_t, vp]
        L.ccj_gen_uniform_keys.argtypes = [vp, u64, u64, u64, u64, vp]
        L.ccj_gen_reference_keys.argtypes = [vp, u64, u64, u64, u64, vp]
        L.ccj_gen_c3_keys.argtypes = [vp, u64, u64, u64, u64, u64, C.c_uint32, vp]
        L.ccj_probe_cost.argtypes = [vp, vp, u64, vp, vp]
        L.ccj_probe_cost_walk.argtypes = [vp, vp, u64, vp, vp]
        L.ccj_set_phase_events.argtypes = [C.POINTER(vp), C.c_uint32]
        L.ccj_probe_visits.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp, vp]
        L.ccj_compact_workspace_size.restype = C.c_size_t
        L.ccj_compact_workspace_size.argtypes = [u64, u64, C.c_uint32, C.c_uint32, C.c_uint32]
        L.ccj_compact.argtypes = [C.POINTER(CompactArgs), vp]
        L.ccj_partition_workspace_size.restype = C.c_size_t
        L.ccj_partition_workspace_size.argtypes = [u64, C.c_uint32]
        L.ccj_partition_by_owner.argtypes = [vp, u64, C.c_uint32, u64, vp, vp, vp, vp, C.c_size_t, vp]
        L.ccj_result_checksum_mapped.argtypes = [vp, vp, vp, u64, u64, C.c_uint32, vp, vp, vp]
        L.ccj_result_checksum.argtypes = [vp, vp, vp, u64, u64, C.c_uint32, u64, vp, vp]
        L.ccj_partition_by_owner_fixed.argtypes = [vp, u64, C.c_uint32, C.c_uint32, u64, vp, vp, vp, vp, vp,
                                                   C.c_size_t, vp]
        L.ccj_segment_chunk_counts.argtypes = [vp, C.c_uint32, u64, C.c_uint32, vp, vp, vp]
        L.ccj_partition_grouped_workspace_size.argtypes = [C.c_uint32]
        L.ccj_partition_grouped_workspace_size.restype = C.c_size_t
        L.ccj_partition_grouped_sub_cap.argtypes = [u64, C.c_uint32, C.c_uint32]
        L.ccj_partition_grouped_sub_cap.restype = u64
        L.ccj_partition_by_owner_grouped.argtypes = [vp, u64, C.c_uint32, C.c_uint32, u64, C.c_uint32, vp, vp, vp, vp, vp,
                                                     C.c_size_t, vp]
        L.ccj_pipeline_create.argtypes = [C.POINTER(vp), C.c_uint32, C.c_uint32, i32, C.POINTER(vp)]
        L.ccj_pipeline_run.argtypes = [vp, C.POINTER(vp), u64, vp, C.POINTER(PipelineResult)]
        L.ccj_pipeline_free.argtypes = [vp]
        L.ccj_pipeline_set_thresholds.argtypes = [vp, vp]
        L.ccj_pipeline_checksum.argtypes = [C.POINTER(PipelineResult), C.c_uint32, vp, vp]
        L.ccj_stream_create_cu_masked.argtypes = [C.POINTER(C.c_uint32), C.c_uint32, C.POINTER(vp)]
        L.ccj_stream_destroy.argtypes = [vp]
        L.ccj_device_cus.argtypes = [C.POINTER(C.c_uint32)]
        L.ccj_copy_device.argtypes = [vp, vp, u64, vp]
        _lib = L
    return _lib


def source_hash() -> str:
    """The build hash (Makefile SRC_HASH) of the sources in this tree: SHA-256 of csrc/*.hip and
    csrc/*.h in sorted path order, then include/ccj.h, as 16 hex digits."""
    import glob
    import hashlib
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")) + glob.glob(os.path.join(HERE, "csrc", "*.h")))
    for f in files + [os.path.join(HERE, "..", "include", "ccj.h")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_hash() -> str:
    """The build hash compiled into the loaded library (ccj_build_hash)."""
    return lib().ccj_build_hash().decode()


def last_gather_kernel() -> str:
    """The payload-gather kernel this thread's last probe with payload columns ran."""
    return lib().ccj_last_gather_kernel().decode()


def check(rc: int, what: str):
    if rc != 0:
        raise CCJError(f"{what} failed ({rc}): {lib().ccj_last_error().decode()}")


def _stream(stream):
    """HIP stream handle for a library call.  Work queued on the caller's current stream (tensor
    allocations, copies) is ordered before the call when `stream` is a different stream."""
    import torch
    cur = torch.cuda.current_stream()
    if stream is None:
        return C.c_void_p(cur.cuda_stream)
    if stream != cur:
        stream.wait_stream(cur)
    return C.c_void_p(stream.cuda_stream)


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class PhaseEvents:
    """One probe call's phase boundaries in the reference's 4-phase schema (CycleProfiler,
    profiler.h:262-290), timed by HIP events the library records at its kernel boundaries
    (ccj_set_phase_events): [0] start, [1] hash & find bucket done, [2] match + advance done,
    [3] gather done.  arm() before the call (this thread's next probe calls record them), ms()
    after the stream has finished: (hash_find, match_advance, gather) in ms."""

    def __init__(self):
        h = _hip()
        self.ev = [C.c_void_p() for _ in range(4)]
        for e in self.ev:
            if h.hipEventCreate(C.byref(e)) != 0:
                raise CCJError("hipEventCreate failed")

    _armed = None  # the instance whose events the library holds (one-shot: the next probe call clears them)

    def arm(self):
        arr = (C.c_void_p * 4)(*[e.value for e in self.ev])
        check(lib().ccj_set_phase_events(arr, 4), "ccj_set_phase_events")
        PhaseEvents._armed = id(self)

    @staticmethod
    def disarm():
        check(lib().ccj_set_phase_events(None, 0), "ccj_set_phase_events")
        PhaseEvents._armed = None

    def ms(self):
        h = _hip()
        out = []
        for a, b in zip(self.ev[:-1], self.ev[1:]):
            t = C.c_float(0.0)
            if h.hipEventElapsedTime(C.byref(t), a, b) != 0:
                raise CCJError("hipEventElapsedTime failed (phase events not recorded?)")
            out.append(float(t.value))
        return tuple(out)

    def __del__(self):
        try:
            if PhaseEvents._armed == id(self):  # never leave the library holding destroyed events
                PhaseEvents.disarm()
            for e in self.ev:
                _hip().hipEventDestroy(e)
        except Exception:
            pass


def device_init(device: int = 0):
    check(lib().ccj_device_init(device), "ccj_device_init")


def gen_uniform_keys(n: int, seed: int, rng: int, first_row: int = 0, out=None, stream=None):
    """Device column of SplitMix64 keys (oracle/ccj_gen.h ccj_uniform_key stream)."""
    import torch
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=torch.device("cuda", torch.cuda.current_device()))
    check(lib().ccj_gen_uniform_keys(_ptr(out), n, seed, first_row, rng, _stream(stream)), "ccj_gen_uniform_keys")
    return out


def result_checksum(out, chunk: int, row_base: int = 0, row_map=None, stream=None):
    """(matches, L2 checksum) of a probe output, computed on the device.  row_map: optional device
    uint64 column giving the global row of every probed position (shuffled inputs)."""
    import torch
    acc = torch.zeros(2, dtype=torch.int64, device=out["count"].device)
    if row_map is None:
        check(lib().ccj_result_checksum(_ptr(out["count"]), _ptr(out["sel"]), _ptr(out["payload"]), out["n_chunks"],
                                        out["cap"], chunk, row_base, _ptr(acc), _stream(stream)), "ccj_result_checksum")
    else:
        check(lib().ccj_result_checksum_mapped(_ptr(out["count"]), _ptr(out["sel"]), _ptr(out["payload"]),
                                               out["n_chunks"], out["cap"], chunk, _ptr(row_map), _ptr(acc),
                                               _stream(stream)), "ccj_result_checksum_mapped")
    torch.cuda.synchronize()
    m, l2 = acc.cpu().tolist()
    return m, l2 & 0xFFFFFFFFFFFFFFFF


def gen_c3_keys(n: int, seed: int, n_build: int, cf: int = 1, hit_ppm: int = 100000, first_row: int = 0,
                out=None, stream=None):
    """Device C3 probe column (Zipf-skewed hits at hit_ppm / 1e6, misses never match)."""
    import torch
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=torch.device("cuda", torch.cuda.current_device()))
    check(lib().ccj_gen_c3_keys(_ptr(out), n, seed, first_row, n_build, cf, hit_ppm, _stream(stream)),
          "ccj_gen_c3_keys")
    return out


def gen_reference_keys(first: int, n: int, n_total: int, cf: int = 1, out=None, stream=None):
    """Device build-side keys first..first+n-1 of the reference generator (linear_probing_ht.cpp:14-25)."""
    import torch
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=torch.device("cuda", torch.cuda.current_device()))
    check(lib().ccj_gen_reference_keys(_ptr(out), first, n, n_total, cf, _stream(stream)), "ccj_gen_reference_keys")
    return out


class Table:
    def __init__(self, handle: C.c_void_p):
        self._h = handle
        info = TableInfo()
        check(lib().ccj_table_get_info(handle, C.byref(info)), "ccj_table_get_info")
        self.kind, self.layout = info.kind, info.layout
        self.n_keys, self.size = info.n_keys, info.size
        self.max_dup, self.max_rounds = info.max_dup, info.max_rounds
        self.d_table, self.d_bucket_off = info.d_table, info.d_bucket_off

    @classmethod
    def reference(cls, kind: int, n: int, cf: int = 1, layout: int = LAYOUT_REFERENCE, stream=None):
        h = C.c_void_p()
        check(lib().ccj_table_build_reference(kind, n, cf, layout, _stream(stream), C.byref(h)),
              "ccj_table_build_reference")
        return cls(h)

    @classmethod
    def from_host(cls, kind: int, keys):
        import numpy as np
        keys = np.ascontiguousarray(keys, dtype=np.int64)
        h = C.c_void_p()
        check(lib().ccj_table_build_from_host(kind, keys.ctypes.data_as(C.c_void_p), len(keys), C.byref(h)),
              "ccj_table_build_from_host")
        return cls(h)

    @classmethod
    def on_device(cls, kind: int, d_keys, stream=None):
        h = C.c_void_p()
        check(lib().ccj_table_build_on_device(kind, _ptr(d_keys), d_keys.numel(), _stream(stream), C.byref(h)),
              "ccj_table_build_on_device")
        return cls(h)

    def free(self):
        if self._h:
            lib().ccj_table_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def arrays(self):
        """The table's device arrays copied to the host (numpy; ccj_table_get_arrays): table
        (slots / chain keys), row, and for chaining off, bucket16 (int64 pairs), bucket8 (or None)."""
        import numpy as np
        import torch
        a = TableArrays()
        check(lib().ccj_table_get_arrays(self._h, C.byref(a)), "ccj_table_get_arrays")
        torch.cuda.synchronize()

        def get(ptr, n, dt):
            return _d2h_bytes(ptr, n * np.dtype(dt).itemsize).view(dt)

        out = dict(table=get(a.d_table, a.positions, np.int64), row=get(a.d_row, a.positions, np.uint32))
        if self.kind == CHAIN:
            out["off"] = get(a.d_bucket_off, self.size + 1, np.uint32)
            out["bucket16"] = get(a.d_bucket16, 2 * self.size, np.int64)
            out["bucket8"] = get(a.d_bucket8, a.n_bucket8, np.uint64) if a.d_bucket8 else None
            out["filter"] = get(a.d_bucket_filter, a.n_filter_words, np.uint32) if a.d_bucket_filter else None
        return out

    def set_payload(self, d_payload, n_cols: int, stream=None):
        """Attach build payload columns: d_payload row-major int64 [n_keys, n_cols] in build order."""
        check(lib().ccj_table_set_payload(self._h, _ptr(d_payload), n_cols, _stream(stream)), "ccj_table_set_payload")
        self.n_payload_cols = n_cols

    def build_rank_index(self, stream=None):
        """The rank walk's window index (ccj_table_build_rank_index; CCJ_PART_RANK needs it).  Only
        libccj_tuning.so contains the rank walk: libccj.so refuses with CCJ_ERR_INVALID."""
        check(lib().ccj_table_build_rank_index(self._h, _stream(stream)), "ccj_table_build_rank_index")

    def probe_cost(self, keys, stream=None):
        """(table words examined, matches) over a key column — roofline accounting."""
        import torch
        acc = torch.zeros(2, dtype=torch.int64, device=keys.device)
        check(lib().ccj_probe_cost(self._h, _ptr(keys), keys.numel(), _ptr(acc), _stream(stream)), "ccj_probe_cost")
        torch.cuda.synchronize()
        a = acc.cpu().tolist()
        return a[0], a[1]

    def probe_cost_walk(self, keys, stream=None):
        """(words examined, matches, words a first-match walk examines, its aligned 32-byte windows)
        over a key column (ccj_probe_cost_walk) — roofline accounting of the first-match walk."""
        import torch
        acc = torch.zeros(4, dtype=torch.int64, device=keys.device)
        check(lib().ccj_probe_cost_walk(self._h, _ptr(keys), keys.numel(), _ptr(acc), _stream(stream)),
              "ccj_probe_cost_walk")
        torch.cuda.synchronize()
        return tuple(int(x) for x in acc.cpu().tolist())

    def alloc_outputs(self, n_rows: int, chunk: int, cap: int | None = None, rounds: bool = True,
                      payload: bool = True, device=None, pos: bool = False, payload_cols: int = 0):
        import torch
        dev = device or torch.device("cuda", torch.cuda.current_device())
        n_chunks = (n_rows + chunk - 1) // chunk
        cap = cap if cap is not None else chunk * max(1, int(self.max_dup))
        mr = max(1, int(self.max_rounds)) + 1 if rounds else 0
        o = dict(
            cap=cap, max_rounds=mr, n_chunks=n_chunks,
            count=torch.empty(n_chunks, dtype=torch.int32, device=dev),
            sel=torch.empty(n_chunks * cap, dtype=torch.int32, device=dev),
            payload=torch.empty(n_chunks * cap, dtype=torch.int64, device=dev) if payload else None,
            rounds=torch.empty(n_chunks, dtype=torch.int32, device=dev) if rounds else None,
            round_counts=torch.zeros(n_chunks * mr, dtype=torch.int32, device=dev) if rounds else None,
            status=torch.zeros(1, dtype=torch.int32, device=dev),
            pos=torch.empty(n_chunks * cap, dtype=torch.int32, device=dev) if pos else None,
            payload_cols=[torch.empty(n_chunks * cap, dtype=torch.int64, device=dev) for _ in range(payload_cols)],
        )
        return o

    def partitioned_positions(self, n_rows: int, chunk: int) -> int:
        """Positions of the partitioned column layout (row-map entries; outputs hold
        positions / chunk chunks) — ccj_probe_partitioned_positions."""
        return int(lib().ccj_probe_partitioned_positions(self._h, n_rows, chunk))

    def alloc_partitioned(self, n_rows: int, chunk: int, device=None):
        """Workspace + row map for probe_partitioned."""
        import torch
        dev = device or torch.device("cuda", torch.cuda.current_device())
        ws_bytes = lib().ccj_probe_partitioned_workspace_size(self._h, n_rows, chunk)
        positions = self.partitioned_positions(n_rows, chunk)
        return dict(ws=torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=dev), ws_bytes=ws_bytes,
                    row_map=torch.empty(max(positions, 1), dtype=torch.int32, device=dev), positions=positions,
                    n_rows=n_rows, chunk=chunk)

    def probe_partitioned(self, keys, chunk: int, out=None, part=None, stream=None, exact: bool = False,
                          retry: bool = True, counts=None, rows: bool = False, rank: bool = False,
                          share: bool = False, **alloc_kw):
        """Slot-range-partitioned probe (ccj_probe_partitioned): L1/L2 results of probe(); out_sel
        indexes the partitioned layout and part["row_map"] maps a live position back to its row.
        The default one-pass split may overflow a segment under heavy key skew
        (FLAG_PART_OVERFLOW); with retry=True that is checked (one stream synchronisation) and the
        probe re-run with the exact split, as the ABI prescribes.  counts: live rows per input chunk
        (fixed-capacity segments, e.g. the multi-GPU exchange's receive buffers); with counts an
        overflow is left to the caller (the exact split takes no counts).  rows=True
        (CCJ_PART_ROWS: LP, distinct keys, cap == chunk): out_sel holds the original row of every
        match instead of its position (result_checksum(out, 0) then needs no row map).
        rank=True (CCJ_PART_RANK): the rank walk where it applies (LP, distinct keys, cap == chunk)."""
        n = keys.numel()
        if rank and part is None:
            self.build_rank_index(stream)  # before the workspace is sized (it grows with the index)
        if part is None:
            part = self.alloc_partitioned(n, chunk)
        if part["n_rows"] != n or part["chunk"] != chunk:
            raise CCJError("partition workspace was sized for another column / chunk")
        if out is None:
            alloc_kw.setdefault("rounds", False)
            out = self.alloc_outputs(part["positions"], chunk, **alloc_kw)
        n_chunks = (part["positions"] + chunk - 1) // chunk
        if out["count"].numel() < n_chunks or out["sel"].numel() < n_chunks * out["cap"]:
            raise CCJError("probe output buffers smaller than the partitioned layout needs")
        a = self._args(keys, chunk, None, counts, out)
        a.out_round_counts = None  # no Next boundaries in partition order
        sw = (PART_RANK if rank else 0) | (PART_SHARE if share else 0)
        flags = (PART_EXACT if exact else 0) | (PART_ROWS if rows else 0) | sw
        row_map = None if rows else _ptr(part["row_map"])
        check(lib().ccj_probe_partitioned(self._h, C.byref(a), flags, row_map, _ptr(part["ws"]),
                                          part["ws_bytes"], _stream(stream)), "ccj_probe_partitioned")
        if retry and not exact and counts is None:
            import torch
            if stream is not None:
                stream.synchronize()
            else:
                torch.cuda.synchronize()
            st = int(out["status"].item())
            if st & FLAG_PART_OVERFLOW:
                out["status"].fill_(st & ~FLAG_PART_OVERFLOW)
                torch.cuda.synchronize()  # the fill ran on torch's stream, the re-run goes on `stream`
                check(lib().ccj_probe_partitioned(self._h, C.byref(a), PART_EXACT | (PART_ROWS if rows else 0) | sw,
                                                  row_map, _ptr(part["ws"]), part["ws_bytes"], _stream(stream)),
                      "ccj_probe_partitioned")
                out["exact_retry"] = True
        out["n_chunks"] = n_chunks
        out["row_map"] = None if rows else part["row_map"]
        out["rows_in_sel"] = rows
        return out

    def _args(self, keys, chunk, sel, counts, out):
        # host-side shape checks: the kernel trusts these sizes (no out-of-bounds reads/writes)
        n_chunks = (keys.numel() + chunk - 1) // chunk
        if counts is not None and counts.numel() < n_chunks:
            raise CCJError(f"counts has {counts.numel()} entries for {n_chunks} chunks")
        if sel is not None and sel.numel() < (n_chunks * chunk if counts is not None else keys.numel()):
            raise CCJError("sel shorter than the chunked key column")
        if out["count"].numel() < n_chunks or out["sel"].numel() < n_chunks * out["cap"]:
            raise CCJError("probe output buffers smaller than the input needs")
        a = ProbeArgs(keys=_ptr(keys).value, sel=_ptr(sel).value if sel is not None else None,
                      counts=_ptr(counts).value if counts is not None else None, n_rows=keys.numel(), chunk=chunk,
                      max_rounds=out["max_rounds"], cap=out["cap"], out_count=_ptr(out["count"]).value,
                      out_sel=_ptr(out["sel"]).value,
                      out_payload=_ptr(out["payload"]).value if out["payload"] is not None else None,
                      out_rounds=_ptr(out["rounds"]).value if out["rounds"] is not None else None,
                      out_round_counts=_ptr(out["round_counts"]).value if out["round_counts"] is not None else None,
                      status=_ptr(out["status"]).value)
        if out.get("pos") is not None:
            a.out_pos = out["pos"].data_ptr()
        cols = out.get("payload_cols") or []
        a.n_payload_cols = len(cols)
        for i, col in enumerate(cols):
            a.out_payload_cols[i] = col.data_ptr()
        return a

    def alloc_ordered(self, n_rows: int, chunk: int, device=None):
        """Workspace of probe_ordered (None when the table takes ccj_probe's one-pass route)."""
        import torch
        b = lib().ccj_probe_ordered_workspace_size(self._h, n_rows, chunk)
        if b == 0:
            return None
        dev = device or torch.device("cuda", torch.cuda.current_device())
        return dict(ws=torch.empty(b, dtype=torch.uint8, device=dev), ws_bytes=b, n_rows=n_rows, chunk=chunk)

    def probe_ordered(self, keys, chunk: int, counts=None, out=None, ws=None, stream=None, retry: bool = True,
                      **alloc_kw):
        """ccj_probe_ordered: probe()'s reference-order (L3) outputs, through the slot-partitioned
        layout for large LP tables.  With retry=True an overflow of the split (extreme key skew)
        is checked (one stream synchronisation) and the chunk is re-run with probe()."""
        if out is None:
            out = self.alloc_outputs(keys.numel(), chunk, **alloc_kw)
        if ws is None:
            ws = self.alloc_ordered(keys.numel(), chunk)
        a = self._args(keys, chunk, None, counts, out)
        w, wb = (None, 0) if ws is None else (_ptr(ws["ws"]), ws["ws_bytes"])
        check(lib().ccj_probe_ordered(self._h, C.byref(a), w, wb, _stream(stream)), "ccj_probe_ordered")
        if retry and ws is not None:
            import torch
            if stream is not None:
                stream.synchronize()
            else:
                torch.cuda.synchronize()
            st = int(out["status"].item())
            if st & FLAG_PART_OVERFLOW:
                out["status"].fill_(st & ~FLAG_PART_OVERFLOW)
                torch.cuda.synchronize()
                self.probe(keys, chunk, counts=counts, out=out, stream=stream)
                out["exact_retry"] = True
        return out

    def probe_visits(self, keys, sel=None, count: int | None = None, max_rounds: int | None = None, stream=None):
        """ccj_probe_visits: (vals [count, max_rounds] int64, len [count] uint32) — the table value
        row i = keys[sel[i]] visits in each round it stays active (InOneNext's writes)."""
        import torch
        n = int(sel.numel() if sel is not None else keys.numel()) if count is None else int(count)
        mr = int(max_rounds or self.max_rounds + 1)
        vals = torch.zeros((n, mr), dtype=torch.int64, device=keys.device)
        ln = torch.zeros(n, dtype=torch.int32, device=keys.device)
        check(lib().ccj_probe_visits(self._h, _ptr(keys), _ptr(sel) if sel is not None else None, n, mr, _ptr(vals),
                                     _ptr(ln), _stream(stream)), "ccj_probe_visits")
        return vals, ln

    def probe(self, keys, chunk: int, sel=None, counts=None, out=None, stream=None, **alloc_kw):
        """Batched Probe + Next loop (include/ccj.h ccj_probe).  Returns the output dict."""
        if out is None:
            out = self.alloc_outputs(keys.numel(), chunk, **alloc_kw)
        a = self._args(keys, chunk, sel, counts, out)
        check(lib().ccj_probe(self._h, C.byref(a), _stream(stream)), "ccj_probe")
        return out



def compact(probe_out, chunk: int, cols=(), payload: bool = True, rows: bool = True, stream=None,
            threshold: int = 0, key_cols=()):
    """Device compaction of a probe output's Next results (include/ccj.h ccj_compact).

    Returns dict(n_chunks (int), counts, cols [list], payload, row, status) — dense output chunks of
    `chunk` rows in the (fixed) NaiveCompactor order; with threshold T, results of >= T rows pass
    through as their own chunk (0 = chunk: NaiveCompactor).  key_cols: indices of `cols` that are
    the probe's join-key column — filled from the payload (equal on every equi-join match) instead
    of gathered (include/ccj.h ccj_compact_args.key_cols).
    """
    import torch
    dev = probe_out["count"].device
    n_chunks, cap = probe_out["n_chunks"], probe_out["cap"]
    if probe_out.get("round_counts") is None:
        raise CCJError("compact needs the probe's per-round counts (alloc_outputs(rounds=True))")
    out_chunks = (n_chunks * cap + chunk - 1) // chunk + 1
    if 0 < threshold < chunk:  # pass-through chunks are not full: at most one per Next result
        out_chunks += n_chunks * min(probe_out["max_rounds"], cap // threshold + 1)
    out_rows = out_chunks * chunk
    ws_bytes = lib().ccj_compact_workspace_size(n_chunks, cap, chunk, probe_out["max_rounds"], threshold)
    ws = torch.empty(max(ws_bytes, 8), dtype=torch.uint8, device=dev)
    o = dict(
        counts=torch.zeros(out_rows // chunk, dtype=torch.int32, device=dev),
        cols=[torch.empty(out_rows, dtype=torch.int64, device=dev) for _ in cols],
        payload=torch.empty(out_rows, dtype=torch.int64, device=dev) if payload else None,
        row=torch.empty(out_rows, dtype=torch.int64, device=dev) if rows else None,
        n=torch.zeros(1, dtype=torch.int64, device=dev),
        status=torch.zeros(1, dtype=torch.int32, device=dev),
        chunk=chunk,
    )
    a = CompactArgs()
    a.count, a.sel = _ptr(probe_out["count"]).value, _ptr(probe_out["sel"]).value
    a.payload = _ptr(probe_out["payload"]).value if probe_out.get("payload") is not None else None
    a.rounds, a.round_counts = _ptr(probe_out["rounds"]).value, _ptr(probe_out["round_counts"]).value
    a.n_chunks, a.cap, a.max_rounds, a.chunk = n_chunks, cap, probe_out["max_rounds"], chunk
    a.n_cols = len(cols)
    a.threshold = threshold
    a.key_cols = sum(1 << k for k in key_cols)
    for i, col in enumerate(cols):
        a.cols[i] = col.data_ptr() if col is not None else None
        a.out_cols[i] = o["cols"][i].data_ptr()
    a.out_payload = o["payload"].data_ptr() if payload else None
    a.out_row = o["row"].data_ptr() if rows else None
    a.out_chunk_counts = o["counts"].data_ptr()
    a.out_cap_rows = out_rows
    a.out_n_chunks = o["n"].data_ptr()
    a.workspace, a.workspace_bytes = ws.data_ptr(), ws_bytes
    a.status = o["status"].data_ptr()
    o["_ws"] = ws
    check(lib().ccj_compact(C.byref(a), _stream(stream)), "ccj_compact")
    return o


class OwnerPartitioner:
    """Owner partitioning (include/ccj.h ccj_partition_by_owner) with reusable buffers."""

    def __init__(self, n: int, parts: int, device=None):
        import torch
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.n, self.parts = n, parts
        self.ws_bytes = lib().ccj_partition_workspace_size(n, parts)
        self.ws = torch.empty(max(self.ws_bytes, 8), dtype=torch.uint8, device=dev)
        self.keys = torch.empty(n, dtype=torch.int64, device=dev)
        self.rows = torch.empty(n, dtype=torch.int64, device=dev)
        self.counts = torch.zeros(parts, dtype=torch.int64, device=dev)

    def __call__(self, keys, row_base: int = 0, stream=None):
        assert keys.numel() == self.n
        check(lib().ccj_partition_by_owner(_ptr(keys), self.n, self.parts, row_base, _ptr(self.keys),
                                           _ptr(self.rows), _ptr(self.counts), _ptr(self.ws), self.ws_bytes,
                                           _stream(stream)), "ccj_partition_by_owner")
        return self.keys, self.rows, self.counts


class FixedOwnerPartitioner:
    """Fixed-capacity owner partitioning (ccj_partition_by_owner_fixed): destination d's keys and
    u32 rows at [d*seg_cap, d*seg_cap + count_d), so an all-to-all needs no host-side sizes."""

    def __init__(self, n: int, parts: int, seg_cap: int, device=None):
        import torch
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.n, self.parts, self.seg_cap = n, parts, seg_cap
        self.ws_bytes = lib().ccj_partition_workspace_size(n, parts)
        self.ws = torch.empty(max(self.ws_bytes, 8), dtype=torch.uint8, device=dev)

    def __call__(self, keys, row_base, out_keys, out_rows, out_counts, status, stream=None):
        assert keys.numel() == self.n and out_keys.numel() >= self.parts * self.seg_cap
        check(lib().ccj_partition_by_owner_fixed(_ptr(keys), self.n, self.parts, row_base, self.seg_cap,
                                                 _ptr(out_keys), _ptr(out_rows), _ptr(out_counts), _ptr(status),
                                                 _ptr(self.ws), self.ws_bytes, _stream(stream)),
              "ccj_partition_by_owner_fixed")


OWNER_GROUPS = 8  # CCJ_OWNER_GROUPS


class GroupedOwnerPartitioner:
    """One-pass fixed-capacity owner partitioning (ccj_partition_by_owner_grouped): destination d's
    region is OWNER_GROUPS sub-segments of sub_cap slots, sub-segment (s, g) at (s*8 + g)*sub_cap
    holding counts[s*8 + g] rows (u32 row ids row_base + i), s = d — or, with self_last = the
    caller's rank, s = parts - 1 for the own rank and d - (d > self_last) for the peers."""

    def __init__(self, n: int, parts: int, sub_cap: int, device=None, self_last: int = -1):
        import torch
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.n, self.parts, self.sub_cap = n, parts, sub_cap
        self.self_last = self_last if 0 <= self_last < parts else 0xFFFFFFFF
        self.ws_bytes = lib().ccj_partition_grouped_workspace_size(parts)
        self.ws = torch.empty(max(self.ws_bytes, 8), dtype=torch.uint8, device=dev)

    def __call__(self, keys, row_base, out_keys, out_rows, out_counts, status, stream=None):
        assert keys.numel() == self.n and out_keys.numel() >= self.parts * OWNER_GROUPS * self.sub_cap
        assert out_counts.numel() >= self.parts * OWNER_GROUPS
        check(lib().ccj_partition_by_owner_grouped(_ptr(keys), self.n, self.parts, row_base, self.sub_cap,
                                                   self.self_last, _ptr(out_keys), _ptr(out_rows), _ptr(out_counts), _ptr(status),
                                                   _ptr(self.ws), self.ws_bytes, _stream(stream)),
              "ccj_partition_by_owner_grouped")


def grouped_sub_cap(n: int, parts: int, chunk: int) -> int:
    """Sub-segment capacity for GroupedOwnerPartitioner over n uniformly hashed keys."""
    return int(lib().ccj_partition_grouped_sub_cap(n, parts, chunk))


def copy_device(dst, src, stream=None):
    """dst[:] = src (device tensors of equal byte size, a multiple of 16) by ccj_copy_device."""
    nb = src.numel() * src.element_size()
    assert dst.numel() * dst.element_size() == nb
    check(lib().ccj_copy_device(_ptr(dst), _ptr(src), nb, _stream(stream)), "ccj_copy_device")
    return dst


def device_cus() -> int:
    n = C.c_uint32(0)
    check(lib().ccj_device_cus(C.byref(n)), "ccj_device_cus")
    return int(n.value)


def cu_mask_groups(groups, n_cus: int | None = None, period: int = 32):
    """CU mask (list of u32 words) of the CUs i with (i // 8) % period in `groups`: each group is 8
    consecutive CU numbers (one per XCD where HIP deals CU numbers to the XCDs in turn, a
    contiguous eighth of an XCD's CUs otherwise), so a set of groups spreads over all eight XCDs."""
    n_cus = n_cus or device_cus()
    words = [0] * ((n_cus + 31) // 32)
    for i in range(n_cus):
        if (i // 8) % period in groups:
            words[i // 32] |= 1 << (i % 32)
    return words


def cu_masked_stream(mask_words):
    """A torch stream confined to the CUs of `mask_words` (ccj_stream_create_cu_masked); the
    library's persistent kernels launched on it size their grid to those CUs."""
    import torch
    arr = (C.c_uint32 * len(mask_words))(*mask_words)
    h = C.c_void_p()
    check(lib().ccj_stream_create_cu_masked(arr, len(mask_words), C.byref(h)), "ccj_stream_create_cu_masked")
    st = torch.cuda.ExternalStream(h.value)
    st._ccj_handle = h  # destroyed with ccj_stream_destroy by the owner, if ever (streams live per process)
    return st


def segment_chunk_counts(seg_counts, seg_cap: int, chunk: int, out, status, stream=None):
    check(lib().ccj_segment_chunk_counts(_ptr(seg_counts), seg_counts.numel(), seg_cap, chunk, _ptr(out),
                                         _ptr(status), _stream(stream)), "ccj_segment_chunk_counts")
    return out


_HIP = None


def _hip():
    """The HIP runtime (the one libccj.so and torch use) for raw copies and phase events."""
    global _HIP
    if _HIP is None:
        lib()
        _HIP = C.CDLL("libamdhip64.so")
        _HIP.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _HIP.hipEventCreate.argtypes = [C.POINTER(C.c_void_p)]
        _HIP.hipEventElapsedTime.argtypes = [C.POINTER(C.c_float), C.c_void_p, C.c_void_p]
        _HIP.hipEventDestroy.argtypes = [C.c_void_p]
    return _HIP


def _d2h_bytes(ptr, nbytes):
    """Copy nbytes from a raw device pointer the library owns (hipMemcpy; caller synchronised)."""
    import numpy as np
    out = np.empty(nbytes, np.uint8)
    if nbytes == 0:
        return out
    rc = _hip().hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), nbytes, 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise CCJError(f"hipMemcpy failed ({rc})")
    return out


def _d2h_i64(ptr, n):
    """Copy n int64 from a raw device pointer the library owns (hipMemcpy; caller synchronised)."""
    import numpy as np
    out = np.empty(n, np.int64)
    if n == 0:
        return out
    rc = _hip().hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), n * 8, 2)  # hipMemcpyDeviceToHost
    if rc != 0:
        raise CCJError(f"hipMemcpy failed ({rc})")
    return out


class Pipeline:
    """main.cpp's ExecutePipeline / FlushPipelineCache (main.cpp:119-191) over `tables`, join l
    probing column l, with no compaction or the (fixed) NaiveCompactor between joins
    (ccj_pipeline_run, include/ccj.h).  run() returns the result table as device columns."""

    def __init__(self, tables, chunk: int, compact: bool):
        self.tables = list(tables)  # keep the tables alive as long as the pipeline
        self.joins = len(self.tables)
        arr = (C.c_void_p * self.joins)(*[t._h.value for t in self.tables])
        h = C.c_void_p()
        check(lib().ccj_pipeline_create(arr, self.joins, chunk, COMPACT_FULL if compact else COMPACT_NONE,
                                        C.byref(h)), "ccj_pipeline_create")
        self.h = h
        self.res = PipelineResult()

    def run(self, cols, stream=None):
        """cols: `joins` device int64 columns of equal length (the probe side, column-major)."""
        assert len(cols) == self.joins
        n = cols[0].numel()
        arr = (C.c_void_p * self.joins)(*[c.data_ptr() for c in cols])
        self._cols = cols
        check(lib().ccj_pipeline_run(self.h, arr, n, _stream(stream), C.byref(self.res)), "ccj_pipeline_run")
        return self.res

    def set_thresholds(self, thresholds=None):
        """Per-join pass-through thresholds of the compactors (None: NaiveCompactor everywhere)."""
        arr = None if thresholds is None else (C.c_uint32 * self.joins)(*thresholds)
        check(lib().ccj_pipeline_set_thresholds(self.h, arr), "ccj_pipeline_set_thresholds")

    def stats(self):
        r = self.res
        return [dict(chunks_in=r.chunks_in[l], rows_in=r.rows_in[l], rows_out=r.rows_out[l], ms=r.level_ms[l])
                for l in range(self.joins)]

    def result_columns(self):
        """The result table as numpy int64 columns in the sink's column order: the probe columns,
        then per join a zero column (result column m, never written) and its payload."""
        import numpy as np
        import torch
        torch.cuda.synchronize()
        n = self.res.n_out
        out = [_d2h_i64(self.res.cols[j], n) for j in range(self.joins)]
        for l in range(self.joins):
            out.append(np.zeros(n, np.int64))
            out.append(_d2h_i64(self.res.payload[l], n))
        return out

    def checksum(self, stream=None):
        import torch
        acc = torch.zeros(2, dtype=torch.int64, device="cuda")
        check(lib().ccj_pipeline_checksum(C.byref(self.res), self.joins, _ptr(acc), _stream(stream)),
              "ccj_pipeline_checksum")
        a = acc.cpu().tolist()
        return a[0], a[1] & 0xFFFFFFFFFFFFFFFF

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ccj_pipeline_free(self.h)
            self.h = None
