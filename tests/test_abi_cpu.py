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
    assert ccj.lib().ccj_abi_version() == 2


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
    import subprocess
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", ccj.LIB_PATH], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("roc-obj-ls unavailable")
    assert "gfx950" in out.stdout
