"""Shared test helpers: golden fixtures, probe-output views, reference-shaped inputs."""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def known_answers():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        return json.load(f)


def load_trace(name, view):
    with np.load(os.path.join(GOLDEN, f"trace_{name}_{view}.npz")) as z:
        return {k: z[k] for k in z.files}


def trace_inputs(spec, trace):
    """Re-create the probe input of a trace case: keys (SplitMix64 stream), per-chunk sel, counts."""
    from oracle import oracle as O

    B, n = spec["B"], spec["n_probe"]
    assert spec["gen"] == 0
    keys = O.uniform_keys(spec["seed"], 0, n, spec["range"])
    n_chunks = (n + B - 1) // B
    sel = np.zeros(n_chunks * B, np.uint32)
    counts = trace["chunk_counts"].astype(np.uint32)
    off = 0
    for c in range(n_chunks):
        k = int(counts[c])
        sel[c * B:c * B + k] = trace["chunk_sel"][off:off + k]
        off += k
    return keys, sel, counts


def views_from_rounds(count, sel, payload, rounds, round_counts, cap, max_rounds, merged=False):
    """Rebuild the per-Next trace arrays from a probe result (oracle or device).

    rounds view: one Next per probe round (LP Next, linear_probing_ht.cpp:62-115; chaining InOneNext).
    merged view: chaining Next, whose ScanInnerJoin repeats rounds until a match
    (chaining_ht.cpp:82-107): leading empty rounds merge into the next non-empty one and a tail of
    empty rounds becomes one Next returning 0.
    """
    n_chunk, n_rc, m_sel, m_pay = [], [], [], []
    for c in range(len(count)):
        rcs = [int(x) for x in round_counts[c * max_rounds:c * max_rounds + int(rounds[c])]]
        assert sum(rcs) == int(count[c])
        if merged:
            nexts = [x for x in rcs if x > 0]
            if rcs and rcs[-1] == 0:
                nexts.append(0)
        else:
            nexts = rcs
        for x in nexts:
            n_chunk.append(c)
            n_rc.append(x)
        k = int(count[c])
        m_sel.extend(sel[c * cap:c * cap + k].tolist())
        m_pay.extend(payload[c * cap:c * cap + k].tolist())
    return dict(next_chunk=np.array(n_chunk, np.uint32), next_rc=np.array(n_rc, np.uint32),
                match_sel=np.array(m_sel, np.uint32), match_payload=np.array(m_pay, np.int64))


def assert_trace_equal(got, want):
    for k in ("next_chunk", "next_rc", "match_sel", "match_payload"):
        a, b = np.asarray(got[k]), np.asarray(want[k])
        assert a.shape == b.shape, (k, a.shape, b.shape)
        if not np.array_equal(a, b):
            i = int(np.flatnonzero(a != b)[0])
            raise AssertionError(f"{k} differs first at {i}: got {a[i]} want {b[i]}")


def ref_keys(n, cf):
    from oracle import oracle as O
    return O.ref_build_keys(n, cf)


def oracle_pipeline(tables, cols, B, compact, cap_factor, max_rounds=256, thresholds=None):
    """main.cpp's ExecutePipeline / FlushPipelineCache (main.cpp:119-191) restated join by join on
    the oracle (TEST INFRASTRUCTURE): join l probes column l of every input chunk with the
    oracle's L3 probe (round-major Next order), then the Next results, in pipeline order, either
    become the next join's chunks one by one (no compaction) or are re-chunked by the oracle's
    literal NaiveCompactor simulation (compact_plan, compactor.cpp:5-41 with the :36 fix).
    Returns the result table's carried columns (probe columns, then one payload per join) in the
    ResultCollector's append order.  thresholds[l]: join l's compactor lets results of at least
    that many rows pass through (0 = chunk: NaiveCompactor)."""
    from oracle import oracle as O

    carried = [np.asarray(c, np.int64) for c in cols]
    counts = None  # chunk c = rows [c*B, c*B + counts[c]) of the carried arrays
    for l, t in enumerate(tables):
        out = t.probe(carried[l], B, counts=counts, cap_factor=cap_factor, max_rounds=max_rounds)
        cap, R = out["cap"], out["max_rounds"]
        seg_rows, seg_pay, seg_counts = [], [], []
        for c in range(len(out["count"])):
            src = c * cap
            for r in range(int(out["rounds"][c])):
                rc = int(out["round_counts"][c * R + r])
                seg_rows.append(c * B + out["sel"][src:src + rc].astype(np.int64))
                seg_pay.append(out["payload"][src:src + rc])
                seg_counts.append(rc)
                src += rc
        rows = np.concatenate(seg_rows) if seg_rows else np.zeros(0, np.int64)
        pay = np.concatenate(seg_pay) if seg_pay else np.zeros(0, np.int64)
        stream = [c[rows] for c in carried] + [pay]
        if compact:
            thr = thresholds[l] if thresholds is not None else 0
            dest, occ = O.compact_plan(np.array(seg_counts, np.uint32), B, thr)
            nxt = []
            for col in stream:
                a = np.zeros(len(occ) * B, np.int64)
                a[dest.astype(np.int64)] = col
                nxt.append(a)
            carried, counts = nxt, occ.astype(np.uint32)
        else:
            keep = [k for k, n in enumerate(seg_counts) if n]
            starts = np.concatenate([[0], np.cumsum(seg_counts)])
            nxt = [np.zeros(len(keep) * B, np.int64) for _ in stream]
            for i, k in enumerate(keep):
                a, n = starts[k], seg_counts[k]
                for q, col in enumerate(stream):
                    nxt[q][i * B:i * B + n] = col[a:a + n]
            carried, counts = nxt, np.array([seg_counts[k] for k in keep], np.uint32)
        if counts.size == 0:
            return [np.zeros(0, np.int64) for _ in range(len(cols) + len(tables))]
    # result table in append order: chunk by chunk, its first counts[c] rows
    idx = np.concatenate([np.arange(c * B, c * B + int(n)) for c, n in enumerate(counts)])
    return [col[idx] for col in carried]
