"""Roofline work accounting through the C ABI (ccj_probe_cost / ccj_probe_cost_walk) against a
numpy model on small tables: the reference's examined words (LP: home slot through the
terminating empty, linear_probing_ht.cpp:72-110; chaining: the whole chain, chaining_ht.cpp:82-124),
matches, and what a walk that ends a row at its first match examines (words, aligned 32-byte
windows) — the bytes bench.py's `frac_walked` counts."""
import numpy as np
import pytest

from helpers import ref_keys
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import ccj  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ccj.device_init(0)


def model(kind, build, probe):
    size = 1
    while size < (4 * len(build) if kind == ccj.LP else 2 * len(build)):
        size <<= 1
    mask = size - 1
    ex = mt = fw = win = 0
    if kind == ccj.LP:
        slots = [-1] * size
        for k in build:
            s = O.murmurhash64(int(k)) & mask
            while slots[s] != -1:
                s = (s + 1) & mask
            slots[s] = int(k)
        for k in probe:
            h = O.murmurhash64(int(k)) & mask
            s, w, first = h, 0, 0
            while True:
                v = slots[s]
                ex += 1
                w += 1
                if v == -1:
                    break
                if v == k:
                    mt += 1
                    first = first or w
                s = (s + 1) & mask
            L = first or w
            fw += L
            win += ((h & 3) + L - 1) // 4 + 1
    else:
        chains = {}
        for k in build:
            chains.setdefault(O.murmurhash64(int(k)) & mask, []).append(int(k))
        starts, pos = {}, 0
        for b in range(size):  # CSR start of every bucket
            starts[b] = pos
            pos += len(chains.get(b, []))
        for k in probe:
            b = O.murmurhash64(int(k)) & mask
            ch = chains.get(b, [])
            first = 0
            for i, v in enumerate(ch):
                ex += 1
                if v == k:
                    mt += 1
                    first = first or i + 1
            L = first or len(ch)
            fw += L
            lo = starts[b]
            if L > 1:
                win += ((lo + L - 1) >> 1) - ((lo + 1) >> 1) + 1
    return ex, mt, fw, win


@pytest.mark.parametrize("kind", [ccj.LP, ccj.CHAIN])
@pytest.mark.parametrize("cf", [1, 3])
def test_probe_cost_walk_equals_model(kind, cf):
    build = ref_keys(3000, cf)
    probe = O.uniform_keys(13, 0, 20000, 3 * 3000 // cf + 7)
    table = ccj.Table.from_host(kind, build)
    keys = torch.from_numpy(probe).cuda()
    got = table.probe_cost_walk(keys)
    want = model(kind, build, probe)
    assert got == want
    assert table.probe_cost(keys) == want[:2]
    m, _ = O.count_uniform(13, 0, 20000, 3 * 3000 // cf + 7, 3000, cf)
    assert got[1] == m
