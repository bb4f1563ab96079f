#!/usr/bin/env python3
"""Summarise a tools/unit_pass.sh run (gpurun_out/prof_TAG) into profiles/TAG_units.json: per kernel
the raw counters (last dispatch of each pass) and the fractions that name the unit holding it —
busy and stall cycles of the TA / TD / TCP instances (one per CU; GRBM_GUI_ACTIVE is summed over the
8 XCDs, so a fraction = counter / (GRBM_GUI_ACTIVE / 8 x CUs)), the SQ's
wave-cycle split (issuing / waiting at s_waitcnt or a barrier / stalled at issue), LDS bank-conflict
share, and the L1 -> L2 request latency.   usage: tools/unit_summary.py TAG [--cus 256] [--xcds 8]"""
import argparse
import collections
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--xcds", type=int, default=8)
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    raw = collections.defaultdict(dict)
    for d in sorted(os.listdir(src)):
        p = os.path.join(src, d, "pmc_counter_collection.csv")
        if not d.startswith("pmc_") or not os.path.exists(p):
            continue
        grp = {}
        with open(p) as f:
            for r in csv.DictReader(f):
                grp.setdefault(r["Kernel_Name"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        for k, cs in grp.items():
            gui = cs.get("GRBM_GUI_ACTIVE")
            for c, v in cs.items():
                raw[k][c] = v
                if gui and c != "GRBM_GUI_ACTIVE":
                    raw[k][c + "@gui"] = gui  # the pass's own cycle count, for its per-CU fractions
    out = {}
    for k, c in raw.items():
        f = {}

        def per_cu(name):
            if name in c and name + "@gui" in c:
                f[name.replace("_sum", "") + "_frac"] = c[name] / (c[name + "@gui"] / a.xcds * a.cus)
        for n in ("TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum",
                  "TD_TD_BUSY_sum", "TD_TC_STALL_sum", "TCP_TCR_TCP_STALL_CYCLES_sum", "TCP_PENDING_STALL_CYCLES_sum",
                  "TCP_TCP_TA_DATA_STALL_CYCLES_sum", "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"):
            per_cu(n)
        if "GRBM_TA_BUSY" in c and "GRBM_TA_BUSY@gui" in c:
            f["GRBM_TA_BUSY_frac"] = c["GRBM_TA_BUSY"] / c["GRBM_TA_BUSY@gui"]
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM"):
                if n in c:
                    f[n + "_of_wave_cycles"] = c[n] / w
        if c.get("SQ_LDS_IDX_ACTIVE"):
            f["lds_bank_conflict_share"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]
        if c.get("TCP_TCC_READ_REQ_sum"):
            f["l1_l2_read_latency_cycles"] = c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / c["TCP_TCC_READ_REQ_sum"]
        if c.get("TCP_TCC_WRITE_REQ_sum"):
            f["l1_l2_write_latency_cycles"] = c.get("TCP_TCC_WRITE_REQ_LATENCY_sum", 0) / c["TCP_TCC_WRITE_REQ_sum"]
        out[k] = {"fractions": f, "raw": {n: v for n, v in c.items() if not n.endswith("@gui")}}
    dst = os.path.join(ROOT, "profiles", f"{a.tag}_units.json")
    with open(dst, "w") as fh:
        json.dump({"tag": a.tag, "cus": a.cus, "xcds": a.xcds, "kernels": out}, fh, indent=1, sort_keys=True)
    for k, v in out.items():
        print(k[:60], json.dumps({n: round(x, 3) for n, x in v["fractions"].items()}))


if __name__ == "__main__":
    main()
