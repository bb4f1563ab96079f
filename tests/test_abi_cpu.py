"""CPU-side checks of the C-ABI library: it builds, loads, exports every symbol include/ccj.h
declares, and refuses to compute without a GPU (no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

import ccj

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "ccj.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(ccj_[a-z_0-9]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    L = ccj.lib()
    syms = declared_symbols()
    assert "ccj_probe" in syms and "ccj_table_build_reference" in syms
    for s in syms:
        assert hasattr(L, s), f"libccj.so does not export {s}"
    assert set(ccj.EXPORTS) <= set(syms)


def test_abi_version():
    assert ccj.lib().ccj_abi_version() == ccj.ABI_VERSION == 15


def test_build_hash_matches_the_tree():
    """The library was built from the sources in this tree (ccj_build_hash == the hash of csrc/ and
    include/ccj.h): bench.py relies on it to tell a counter profile of this build from a stale one."""
    h = ccj.build_hash()
    assert len(h) == 16 and int(h, 16) >= 0
    assert h == ccj.source_hash()


def test_fails_loudly_without_device():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    rc = ccj.lib().ccj_device_init(0)
    assert rc == -3  # CCJ_ERR_NO_DEVICE
    assert b"device" in ccj.lib().ccj_last_error()
    h = C.c_void_p()
    rc = ccj.lib().ccj_table_build_reference(0, 16, 1, 0, None, C.byref(h))
    assert rc != 0 and not h.value


def test_built_for_gfx950():
    """The library's offload bundle holds gfx950 code objects (the bundle entry id names the
    target), and no other GPU target."""
    import re
    data = open(ccj.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", data))
    assert targets == {b"gfx950"}, targets


def test_new_entry_points_fail_loudly_without_device():
    """Pipeline, tuner-facing and multi-GPU entry points refuse to run without a GPU and report
    bad arguments before touching the device (no CPU fallback anywhere)."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    L = ccj.lib()
    h = C.c_void_p()
    # no tables -> invalid argument, checked before the device
    assert L.ccj_pipeline_create(None, 3, 256, 1, C.byref(h)) == -1 and not h.value
    arr = (C.c_void_p * 1)(None)
    assert L.ccj_pipeline_create(arr, 1, 256, 1, C.byref(h)) == -1  # null table
    assert L.ccj_pipeline_set_thresholds(None, None) == -1
    assert L.ccj_pipeline_free(None) == 0
    assert L.ccj_pipeline_checksum(None, 1, None, None) == -1
    # fixed-capacity partition: argument checks
    assert L.ccj_partition_by_owner_fixed(None, 10, 3, 0, 16, None, None, None, None, None, 0, None) == -1
    assert L.ccj_segment_chunk_counts(None, 1, 100, 64, None, None, None) == -1  # seg_cap % chunk
    assert L.ccj_gen_c3_keys(None, 10, 1, 0, 100, 1, 100000, None) == -1
    assert L.ccj_gen_c3_keys(None, 0, 1, 0, 100, 1, 2000000, None) == -1  # hit_ppm > 1e6
    assert b"" != L.ccj_last_error()


def test_compact_workspace_grows_with_pass_through():
    L = ccj.lib()
    naive = L.ccj_compact_workspace_size(1000, 2048, 2048, 33, 0)
    gated = L.ccj_compact_workspace_size(1000, 2048, 2048, 33, 1)
    assert gated > naive > 0
