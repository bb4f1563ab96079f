"""The C++ operator facade (host/ccj_operators.h) against the reference's own per-Next traces.

tests/native/facade_trace.cpp drives LPHashTable / HashTable + ScanStructure exactly as the
reference's callers drive the reference (Probe, then Next until HasNext() is false) and prints
every Next result; each must equal the trace recorded from the compiled reference
(tests/golden/trace_*, oracle/ref_driver.cpp): LP's Next / InOneNext / SIMD variants and
chaining's InOneNext give one result per round, chaining's Next merges empty rounds
(ScanInnerJoin, chaining_ht.cpp:82-107) — L3, through the drop-in surface itself."""
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
    nc, nr, ms, mp = [], [], [], []
    for line in p.stdout.splitlines():
        t = line.split()
        if t[0] == "N":
            nc.append(int(t[1]))
            nr.append(int(t[2]))
        else:
            ms.append(int(t[1]))
            mp.append(int(t[2]))
    return dict(next_chunk=np.array(nc, np.uint32), next_rc=np.array(nr, np.uint32),
                match_sel=np.array(ms, np.uint32), match_payload=np.array(mp, np.int64))


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("variant", ["next", "inone", "simdnext", "simdinone"])
def test_facade_next_stream_equals_reference(facade_trace, name, variant):
    spec = CASES[name]["spec"]
    merged = spec["kind"] == "chain" and variant in ("next", "simdnext")
    want = load_trace(name, "merged" if merged else "rounds")
    assert_trace_equal(run(facade_trace, spec, variant), want)
