"""Every timing-only ablation of the tuning build (libccj_tuning.so: CCJ_ABLATE, CCJ_OWNER_ABLATE,
CCJ_GATHER_ABLATE; csrc/ccj_tuning.h) run once at a small size on every path that reads it, in ONE
process: the ablations skip or redirect work so their results are wrong by design, but every kernel
must still finish without a fault, and the status word must hold only the flags the ABI defines.
Round 5's only GPU faults came from such an ablation (CCJ_OWNER_ABLATE=0x200000 before
its LDS image was initialised), so each one is pinned here.

Run by tests/test_rank_gpu.py in a child pytest with CCJ_LIB_PATH = the tuning build; the variables
are set in this process's environment (the tuning build reads them with getenv at every launch)."""
import os

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402

KNOWN_FLAGS = 0x1F  # ccj.h: cap / round / bad input / partition overflow / internal (DPP check)
N_BUILD, N_PROBE, CHUNK = 1 << 18, 1 << 21, 2048

# bits read by the probe walks (ProbeParams::ablate), the slot split (its ablate word) and the
# gather; the owner split's (CCJ_OWNER_ABLATE) words below
PROBE_BITS = [0x1, 0x2, 0x10, 0x20, 0x40, 0x80, 0x100, 0x200, 0x400, 0x2000, 0x4000, 0x8000, 0x10000, 0x40000,
              0x100000, 0x200000]
OWNER_BITS = [0x10, 0x20, 0x40, 0x80, 0x2000, 0x100000, 0x200000]


@pytest.fixture(scope="module")
def tables():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert "tuning" in ccj.LIB_PATH, "run with CCJ_LIB_PATH = libccj_tuning.so"
    ccj.device_init(0)
    lp = ccj.Table.reference(ccj.LP, N_BUILD, 1, ccj.LAYOUT_DEVICE)
    bk = ccj.gen_reference_keys(0, N_BUILD, N_BUILD, 1)
    mult = torch.arange(1, 9, dtype=torch.int64, device="cuda")
    lp.set_payload((bk[:, None] * mult[None, :] + (mult[None, :] - 1)).reshape(-1), 8)
    ch = ccj.Table.reference(ccj.CHAIN, N_BUILD, 1, ccj.LAYOUT_DEVICE)
    keys = ccj.gen_uniform_keys(N_PROBE, 42, N_BUILD)
    c3 = ccj.gen_c3_keys(N_PROBE, 42, N_BUILD, 1)
    torch.cuda.synchronize()
    return lp, ch, keys, c3


def run_paths(lp, ch, keys, c3):
    """Every path once; returns {path: status word}."""
    st = {}
    o = lp.probe_partitioned(keys, CHUNK, rows=True, retry=False)
    st["lp_partitioned_rows"] = o["status"]
    o = lp.probe_partitioned(keys, CHUNK, retry=False)
    st["lp_partitioned"] = o["status"]
    o = lp.probe_partitioned(keys, CHUNK, rows=True, retry=False, payload_cols=8, pos=True)
    st["lp_partitioned_payload"] = o["status"]
    o = lp.probe_ordered(keys, CHUNK, retry=False)
    st["lp_ordered"] = o["status"]
    o = lp.probe(keys[: 1 << 18], CHUNK)
    st["lp_chunk"] = o["status"]
    o = ch.probe_partitioned(c3, CHUNK, retry=False)
    st["chain_partitioned"] = o["status"]
    o = ch.probe_ordered(c3, CHUNK, retry=False)
    st["chain_ordered"] = o["status"]
    for parts in (1, 2, 8):
        sub = ccj.grouped_sub_cap(N_PROBE, parts, CHUNK)
        gp = ccj.GroupedOwnerPartitioner(N_PROBE, parts, sub, self_last=parts - 1)
        ok = torch.empty(parts * ccj.OWNER_GROUPS * sub, dtype=torch.int64, device="cuda")
        orow = torch.empty_like(ok, dtype=torch.int32)
        cnt = torch.zeros(parts * ccj.OWNER_GROUPS, dtype=torch.int64, device="cuda")
        s = torch.zeros(1, dtype=torch.int32, device="cuda")
        gp(keys, 0, ok, orow, cnt, s)
        st[f"owner_split_{parts}"] = s
    torch.cuda.synchronize()  # a fault surfaces here
    return {k: int(v.item()) for k, v in st.items()}


@pytest.mark.parametrize("var,bit", [("CCJ_ABLATE", b) for b in PROBE_BITS] +
                         [("CCJ_OWNER_ABLATE", b) for b in OWNER_BITS] + [("CCJ_GATHER_ABLATE", 1)])
def test_ablation_runs_clean(tables, var, bit):
    os.environ[var] = str(bit)
    try:
        st = run_paths(*tables)
    finally:
        del os.environ[var]
    for path, word in st.items():
        assert word & ~KNOWN_FLAGS == 0, (path, hex(word))
    # the same paths without the ablation: nothing left behind (a clean run is status 0 everywhere
    # but the Zipf-skewed C3 split's overflow flag, which the retrying callers act on)
    clean = run_paths(*tables)
    for path, word in clean.items():
        assert word & ~ccj.FLAG_PART_OVERFLOW == 0, (path, hex(word))
