"""The C ABI's argument checks on a device (include/ccj.h: every call returns CCJ_OK or a negative
ccj_status, with the reason in ccj_last_error(); nothing is launched on a refused call).

Each case starts from arguments that work, breaks one of them, and expects CCJ_ERR_INVALID with the
reason the header documents — then the same call with the good arguments still succeeds (no state
is left behind by a refusal).  tests/test_abi_cpu.py covers the no-device refusals."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

INVALID = -1


@pytest.fixture(scope="module")
def env():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)
    lp = ccj.Table.reference(ccj.LP, 1 << 16, 1, ccj.LAYOUT_DEVICE)
    dup = ccj.Table.reference(ccj.LP, 1 << 16, 3, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(1 << 20, 5, 1 << 17)
    torch.cuda.synchronize()
    return lp, dup, keys


def refused(rc, fragment):
    assert rc == INVALID, rc
    msg = ccj.lib().ccj_last_error().decode()
    assert fragment in msg, msg


def probe_args(table, keys, chunk=2048, **kw):
    out = table.alloc_outputs(keys.numel(), chunk, **kw)
    return table._args(keys, chunk, None, None, out), out


@pytest.mark.parametrize("field,value,fragment", [
    ("chunk", 0, "chunk must be 1..2048"),
    ("chunk", 2049, "chunk must be 1..2048"),
    ("max_rounds", 0, "max_rounds == 0"),
    ("out_count", None, "missing buffer"),
    ("out_sel", None, "missing buffer"),
    ("n_payload_cols", 3, "fewer payload columns"),
])
def test_probe_refuses(env, field, value, fragment):
    lp, _, keys = env
    a, _ = probe_args(lp, keys)
    good = getattr(a, field)
    setattr(a, field, value)
    refused(ccj.lib().ccj_probe(lp._h, C.byref(a), None), fragment)
    setattr(a, field, good)
    assert ccj.lib().ccj_probe(lp._h, C.byref(a), None) == 0
    torch.cuda.synchronize()


def test_probe_null_table_and_args(env):
    lp, _, keys = env
    a, _ = probe_args(lp, keys)
    refused(ccj.lib().ccj_probe(None, C.byref(a), None), "null table/args")
    refused(ccj.lib().ccj_probe(lp._h, None, None), "null table/args")


def _partitioned(table, keys, flags=0, rows_in_sel=False, ws_delta=0, counts=None, round_counts=False, sel=False):
    n = keys.numel()
    part = table.alloc_partitioned(n, 2048)
    out = table.alloc_outputs(part["positions"], 2048, rounds=round_counts)
    a = table._args(keys, 2048, None, counts, out)
    if not round_counts:
        a.out_round_counts = None
    if sel:
        a.sel = keys.data_ptr()
    row_map = None if rows_in_sel else part["row_map"].data_ptr()
    return ccj.lib().ccj_probe_partitioned(table._h, C.byref(a), flags, row_map, part["ws"].data_ptr(),
                                           part["ws_bytes"] + ws_delta, None)


def test_probe_partitioned_refuses(env):
    lp, dup, keys = env
    assert _partitioned(lp, keys) == 0
    refused(_partitioned(lp, keys, sel=True), "sel must be NULL")
    refused(_partitioned(lp, keys, flags=1 << 20), "unknown flags")
    refused(_partitioned(lp, keys, ws_delta=-1), "workspace too small")
    refused(_partitioned(lp, keys, round_counts=True), "no round counts")
    counts = torch.full(((keys.numel() + 2047) // 2048,), 2048, dtype=torch.int32, device=keys.device)
    refused(_partitioned(lp, keys, flags=ccj.PART_EXACT, counts=counts), "one-pass split")
    # rows mode needs distinct keys (cap == chunk): a table with max_dup 3 is refused
    refused(_partitioned(dup, keys, flags=ccj.PART_ROWS, rows_in_sel=True), "CCJ_PART_ROWS")
    assert _partitioned(lp, keys, flags=ccj.PART_ROWS, rows_in_sel=True) == 0
    torch.cuda.synchronize()


def test_probe_ordered_refuses_small_workspace():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)
    big = ccj.Table.reference(ccj.LP, 1 << 21, 1, ccj.LAYOUT_DEVICE)  # 2^23 slots: the partitioned route
    keys = ccj.gen_uniform_keys(1 << 20, 9, 1 << 21)
    ws = big.alloc_ordered(keys.numel(), 2048)
    assert ws is not None
    out = big.alloc_outputs(keys.numel(), 2048)
    a = big._args(keys, 2048, None, None, out)
    refused(ccj.lib().ccj_probe_ordered(big._h, C.byref(a), ws["ws"].data_ptr(), ws["ws_bytes"] - 1, None),
            "workspace")
    assert ccj.lib().ccj_probe_ordered(big._h, C.byref(a), ws["ws"].data_ptr(), ws["ws_bytes"], None) == 0
    torch.cuda.synchronize()
    big.free()


def test_compact_refuses(env):
    lp, _, keys = env
    out = lp.probe(keys[:100000], 256)
    col = keys[:100000]
    with pytest.raises(ccj.CCJError, match="chunk must be 1..2048"):
        ccj.compact(out, 4096, cols=[col])
    with pytest.raises(ccj.CCJError, match="key_cols names a column past n_cols"):
        ccj.compact(out, 256, cols=[col], key_cols=[3])
    with pytest.raises(ccj.CCJError, match="key_cols needs payload"):
        ccj.compact(dict(out, payload=None), 256, cols=[col], key_cols=[0], payload=False)
    with pytest.raises(ccj.CCJError, match="null column"):
        ccj.compact(out, 256, cols=[None])
    good = ccj.compact(out, 256, cols=[col], key_cols=[0])
    torch.cuda.synchronize()
    assert int(good["status"].item()) == 0 and int(good["n"].item()) > 0


def test_table_builds_refuse(env):
    L = ccj.lib()
    h = C.c_void_p()
    refused(L.ccj_table_build_reference(ccj.LP, 1000, 0, ccj.LAYOUT_DEVICE, None, C.byref(h)), "bad argument")
    refused(L.ccj_table_build_reference(7, 1000, 1, ccj.LAYOUT_DEVICE, None, C.byref(h)), "bad table kind")
    refused(L.ccj_table_build_reference(ccj.LP, 1000, 1, 9, None, C.byref(h)), "bad layout")
    refused(L.ccj_table_build_from_host(ccj.LP, None, 10, C.byref(h)), "bad argument")
    refused(L.ccj_table_build_on_device(ccj.CHAIN, None, 10, None, C.byref(h)), "bad argument")
    lp, _, _ = env
    with pytest.raises(ccj.CCJError):
        lp.set_payload(torch.zeros(8, dtype=torch.int64, device="cuda"), 0)  # zero columns


def test_owner_partition_refuses(env):
    _, _, keys = env
    with pytest.raises(ccj.CCJError, match="power of two"):
        ccj.OwnerPartitioner(keys.numel(), 3)(keys)
    with pytest.raises(ccj.CCJError, match="power of two"):
        ccj.OwnerPartitioner(keys.numel(), 128)(keys)
    keys_out, rows, counts = ccj.OwnerPartitioner(keys.numel(), 4)(keys)[:3]
    torch.cuda.synchronize()
    assert int(counts.sum().item()) == keys.numel()


def test_key_generators_refuse():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)
    with pytest.raises(ccj.CCJError, match="bad argument"):
        ccj.gen_uniform_keys(100, 1, 0)  # an empty key range
    np.testing.assert_array_equal(ccj.gen_uniform_keys(0, 1, 10).cpu().numpy(), np.zeros(0, np.int64))
