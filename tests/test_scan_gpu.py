"""The hand-written device scan (csrc/ccj_scan.hip) that the compactor, the pipeline, the exact
multisplit and the chaining build take their offsets from: exclusive prefix sums of u64 and u32
arrays, in place and out of place, at sizes around its 2048-value tiles and across two recursion
levels (> 2048^2 values), against torch's cumulative sum.  The scan is an internal C++ routine, not
an ABI entry point: the test binds its symbol in libccj.so directly."""
import ctypes as C

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

SYM = {"u64": "_ZN3ccj18scan_exclusive_u64EPKmPmmS2_PvP12ihipStream_t",
       "u32": "_ZN3ccj18scan_exclusive_u32EPKjPjmS2_PvP12ihipStream_t"}
TEMP = "_ZN3ccj19scan_u64_temp_bytesEm"


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)
    L = ccj.lib()
    for name in SYM.values():
        f = getattr(L, name)
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        f.restype = C.c_int
    getattr(L, TEMP).argtypes = [C.c_uint64]
    getattr(L, TEMP).restype = C.c_size_t
    return L


def run_scan(L, width, x, in_place):
    n = x.numel()
    tmp = torch.empty(max(1, getattr(L, TEMP)(n)), dtype=torch.uint8, device="cuda")
    tot = torch.full((1,), -1, dtype=x.dtype, device="cuda")
    out = x if in_place else torch.full_like(x, -5)
    src = x.clone() if in_place else x
    rc = getattr(L, SYM[width])(x.data_ptr(), out.data_ptr(), n, tot.data_ptr(), tmp.data_ptr(), None)
    assert rc == 0
    torch.cuda.synchronize()
    return src, out, tot


@pytest.mark.parametrize("n", [0, 1, 7, 2047, 2048, 2049, 3 * 2048 + 5, 2048 * 2048, 2048 * 2048 + 1,
                               2048 * 2048 + 4099])
@pytest.mark.parametrize("in_place", [False, True])
def test_scan_u64_equals_cumsum(lib, n, in_place):
    g = torch.Generator(device="cuda").manual_seed(n + 3)
    x = torch.randint(0, 1 << 40, (n,), generator=g, device="cuda", dtype=torch.int64)
    src, out, tot = run_scan(lib, "u64", x, in_place)
    want = torch.cumsum(src, 0) - src
    assert torch.equal(out, want)
    assert int(tot.item()) == int(src.sum().item())


@pytest.mark.parametrize("n", [5, 2049, 2048 * 2048 + 1])
def test_scan_u32_wraps_like_u32(lib, n):
    g = torch.Generator(device="cuda").manual_seed(n)
    x64 = torch.randint(0, 1 << 31, (n,), generator=g, device="cuda", dtype=torch.int64)
    x = x64.to(torch.int32)
    src, out, tot = run_scan(lib, "u32", x, False)
    want = ((torch.cumsum(x64, 0) - x64) & 0xFFFFFFFF).to(torch.int64)
    assert torch.equal(out.to(torch.int64) & 0xFFFFFFFF, want)
    assert (int(tot.item()) & 0xFFFFFFFF) == (int(x64.sum().item()) & 0xFFFFFFFF)
