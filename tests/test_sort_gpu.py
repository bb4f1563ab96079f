"""The hand-written stable LSD radix sort (csrc/ccj_sort.hip) that the chaining build orders its
tuples by bucket with (chaining_ht.cpp:29-35 appends in generator order, so equal
buckets must keep input order) and that max_dup sorts a key copy with.  Checked against numpy's
stable argsort: (key, value) pairs at sizes around the 4096-key tiles, the C3 bucket width (27 bits),
all-equal keys (every pass skipped), keys with one varying byte, and 64-bit keys with negative
values (sorted as bit patterns).  Internal C++ routines, not ABI entry points: the test binds their
symbols in libccj.so directly, as test_scan_gpu.py does for the scan."""
import ctypes as C

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

PAIRS = "_ZN3ccj20radix_sort_pairs_u32EPjS0_S0_S0_mjPvP12ihipStream_tPb"
KEYS = "_ZN3ccj19radix_sort_keys_u64EPmS0_mPvP12ihipStream_tPb"
TEMP = "_ZN3ccj21radix_sort_temp_bytesEm"


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)
    L = ccj.lib()
    f = getattr(L, PAIRS)
    f.argtypes = [C.c_void_p] * 4 + [C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p, C.POINTER(C.c_bool)]
    f.restype = C.c_int
    f = getattr(L, KEYS)
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.POINTER(C.c_bool)]
    f.restype = C.c_int
    getattr(L, TEMP).argtypes = [C.c_uint64]
    getattr(L, TEMP).restype = C.c_size_t
    return L


def sort_pairs(L, keys, end_bit):
    n = len(keys)
    k = torch.from_numpy(keys.view(np.int32)).cuda()
    v = torch.arange(n, dtype=torch.int32, device="cuda")
    k2, v2 = torch.full_like(k, -7), torch.full_like(v, -7)
    tmp = torch.empty(getattr(L, TEMP)(n), dtype=torch.uint8, device="cuda")
    alt = C.c_bool(False)
    rc = getattr(L, PAIRS)(k.data_ptr(), k2.data_ptr(), v.data_ptr(), v2.data_ptr(), n, end_bit, tmp.data_ptr(), None,
                           C.byref(alt))
    assert rc == 0
    torch.cuda.synchronize()
    ko, vo = (k2, v2) if alt.value else (k, v)
    return ko.cpu().numpy().view(np.uint32), vo.cpu().numpy().view(np.uint32)


def case_keys(name, n):
    g = np.random.default_rng(n + len(name))
    if name == "random27":
        return g.integers(0, 1 << 27, n, dtype=np.uint32), 27
    if name == "few":  # many equal keys per tile: long stable runs
        return g.integers(0, 5, n, dtype=np.uint32), 3
    if name == "equal":  # every pass skipped: input order is the answer
        return np.full(n, 1234, np.uint32), 27
    if name == "one_byte":  # only bits 8-15 vary: one pass
        return (g.integers(0, 256, n, dtype=np.uint32) << 8) | 3, 20
    if name == "descending":
        return np.arange(n, dtype=np.uint32)[::-1].copy() & ((1 << 17) - 1), 17
    raise ValueError(name)


@pytest.mark.parametrize("n", [2, 63, 4095, 4096, 4097, 3 * 4096 + 17, 1 << 20, (1 << 22) + 5])
@pytest.mark.parametrize("name", ["random27", "few", "equal", "one_byte", "descending"])
def test_radix_sort_pairs_is_stable(lib, n, name):
    keys, end_bit = case_keys(name, n)
    got_k, got_v = sort_pairs(lib, keys, end_bit)
    order = np.argsort(keys, kind="stable").astype(np.uint32)
    assert np.array_equal(got_v, order)
    assert np.array_equal(got_k, keys[order])


def test_radix_sort_pairs_sorts_only_the_low_bits(lib):
    """end_bit = 12: keys equal in bits [0, 12) keep input order whatever their high bits."""
    g = np.random.default_rng(5)
    keys = g.integers(0, 1 << 30, 50000, dtype=np.uint32)
    got_k, got_v = sort_pairs(lib, keys, 12)
    order = np.argsort(keys & 0xFFF, kind="stable").astype(np.uint32)
    assert np.array_equal(got_v, order)


@pytest.mark.parametrize("n", [2, 5000, 1 << 21])
def test_radix_sort_keys_u64(lib, n):
    g = np.random.default_rng(n)
    keys = g.integers(-(1 << 62), 1 << 62, n, dtype=np.int64)
    keys[::7] = -1
    keys[1::11] = 12345
    k = torch.from_numpy(keys).cuda()
    k2 = torch.empty_like(k)
    tmp = torch.empty(getattr(lib, TEMP)(n), dtype=torch.uint8, device="cuda")
    alt = C.c_bool(False)
    assert getattr(lib, KEYS)(k.data_ptr(), k2.data_ptr(), n, tmp.data_ptr(), None, C.byref(alt)) == 0
    torch.cuda.synchronize()
    got = (k2 if alt.value else k).cpu().numpy().view(np.uint64)
    assert np.array_equal(got, np.sort(keys.view(np.uint64)))
