"""The C++ operator facade (host/ccj_operators.h) against the reference's own per-Next traces.

tests/native/facade_trace.cpp drives LPHashTable / HashTable + ScanStructure exactly as the
reference's callers drive the reference (Probe, then Next until HasNext() is false) and prints
every Next result; each must equal the trace recorded from the compiled reference
(tests/golden/trace_*, oracle/ref_driver.cpp): LP's Next / InOneNext / SIMD variants and
chaining's InOneNext give one result per round, chaining's Next merges empty rounds
(ScanInnerJoin, chaining_ht.cpp:82-107) — L3, through the drop-in surface itself.  The whole
physical result column m+1 is compared after every call too (trace_*_phys.npz), which covers the
InOneNext variants' writes to unmatched active rows."""
import os
import subprocess

import numpy as np
import pytest

from helpers import assert_trace_equal, known_answers, load_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "chunk-compaction-in-vectorized-execution-simd_amd")
CASES = known_answers()["trace_cases"]

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def facade_trace(tmp_path_factory):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = str(tmp_path_factory.mktemp("facade") / "facade_trace")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(PKG, "host"), "-o", exe, os.path.join(ROOT, "tests", "native", "facade_trace.cpp"),
                    os.path.join(PKG, "host", "ccj_operators.cpp"), "-L", PKG, "-lccj", f"-Wl,-rpath,{PKG}"],
                   check=True)
    return exe


def run(exe, spec, variant):
    args = [exe, spec["kind"], variant, spec["B"], spec["n_build"], spec["cf"], spec["n_probe"], spec["range"],
            spec["seed"], spec["selmode"]]
    p = subprocess.run([str(a) for a in args], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    nc, nr, ms, mp, ph = [], [], [], [], []
    for line in p.stdout.splitlines():
        t = line.split()
        if t[0] == "N":
            nc.append(int(t[1]))
            nr.append(int(t[2]))
        elif t[0] == "P":
            ph.append(int(t[1]))
        else:
            ms.append(int(t[1]))
            mp.append(int(t[2]))
    return dict(next_chunk=np.array(nc, np.uint32), next_rc=np.array(nr, np.uint32),
                match_sel=np.array(ms, np.uint32), match_payload=np.array(mp, np.int64)), np.array(ph, np.uint64)


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("variant", ["next", "inone", "simdnext", "simdinone"])
def test_facade_next_stream_equals_reference(facade_trace, name, variant):
    spec = CASES[name]["spec"]
    merged = spec["kind"] == "chain" and variant in ("next", "simdnext")
    want = load_trace(name, "merged" if merged else "rounds")
    got, phys = run(facade_trace, spec, variant)
    assert_trace_equal(got, want)
    # every physical row of result column m+1 after every Next call: InOneNext / SIMDInOneNext also
    # write the visited slot / chain key of unmatched active rows (linear_probing_ht.cpp:133,
    # chaining_ht.cpp:156), Next / SIMDNext only the matches
    want_phys = np.load(os.path.join(ROOT, "tests", "golden", f"trace_{name}_phys.npz"))[variant]
    assert np.array_equal(phys, want_phys)


def _visit_model(kind, n, cf, keys, sel):
    """Pure-Python restatement (small tables only) of what InOneNext visits per round: LP — the
    non-empty run from the home slot (linear_probing_ht.cpp:4-37 layout, :125-141 walk); chaining —
    the bucket's list in push_back order (chaining_ht.cpp:4-36, :148-163)."""
    from oracle import oracle as O
    build = [int(k) for k in O.ref_build_keys(n, cf)]
    size = 1
    while size < (4 * n if kind == "lp" else 2 * n):
        size <<= 1
    mask = size - 1
    if kind == "lp":
        slots = [-1] * size
        for k in build:
            s = O.murmurhash64(k) & mask
            while slots[s] != -1:
                s = (s + 1) & mask
            slots[s] = k
    else:
        lists = {}
        for k in build:
            lists.setdefault(O.murmurhash64(k) & mask, []).append(k)
    out = []
    for i in sel:
        h = O.murmurhash64(int(keys[i])) & mask
        if kind == "lp":
            v = []
            while slots[(h + len(v)) & mask] != -1:
                v.append(slots[(h + len(v)) & mask])
        else:
            v = lists.get(h, [])
        out.append(v)
    return out


@pytest.mark.parametrize("kind,n,cf", [("lp", 4096, 1), ("lp", 4096, 64), ("chain", 4096, 4), ("chain", 5, 3)])
def test_probe_visits_equals_model(kind, n, cf):
    """ccj_probe_visits through the C ABI: every row's per-round visited values and its active
    round count, against the pure-Python model, with a ragged reversed selection."""
    import torch
    import ccj
    from oracle import oracle as O
    ccj.device_init(0)
    t = ccj.Table.reference(ccj.LP if kind == "lp" else ccj.CHAIN, n, cf)
    keys = O.uniform_keys(9, 0, 2048, 2 * n).astype(np.int64)
    sel = np.arange(1999, -1, -1, dtype=np.int32)[::3].copy()  # 667 rows, reversed, strided
    vals, ln = t.probe_visits(torch.from_numpy(keys).cuda(), torch.from_numpy(sel).cuda())
    torch.cuda.synchronize()
    vals, ln = vals.cpu().numpy(), ln.cpu().numpy()
    want = _visit_model(kind, n, cf, keys, sel)
    assert vals.shape[1] == t.max_rounds + 1
    for i, v in enumerate(want):
        assert ln[i] == len(v), i
        assert vals[i, :len(v)].tolist() == v, i
