#!/usr/bin/env python3
"""Table of a tools/pmc_ab.sh run: per variant, the last dispatch's counters of the kernel, plus
derived per-CU rates (usage: tools/pmc_ab_summary.py TAG [--rows N])."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
rows = float(sys.argv[sys.argv.index("--rows") + 1]) if "--rows" in sys.argv else float(1 << 30)
base = os.path.join(ROOT, "gpurun_out", f"pmcab_{tag}")
out = {}
for vd in sorted(glob.glob(os.path.join(base, "v*"))):
    env = open(os.path.join(vd, "env")).read().strip()
    c = {}
    for p in glob.glob(os.path.join(vd, "*", "pmc_counter_collection.csv")):
        last = {}
        for r in csv.DictReader(open(p)):
            last.setdefault(r["Kernel_Name"], {})[r["Counter_Name"]] = float(r["Counter_Value"])
        for k, v in last.items():
            c.update(v)
    d = dict(c)
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8 or None
    if cyc:
        d["per_row"] = {k: c[k] / rows for k in c if k.startswith(("SQ_INSTS", "TCC_REQ", "TCC_EA0_RD", "TCP_TCC_READ_REQ_sum"))}
        for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum", "TCP_PENDING_STALL_CYCLES_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum"):
            if k in c:
                d[k + "_frac"] = c[k] / cyc / 256
        if "TCP_TCC_READ_REQ_LATENCY_sum" in c and c.get("TCP_TCC_READ_REQ_sum"):
            d["read_latency_cyc"] = c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"]
            d["reads_in_flight_per_cu"] = c["TCP_TCC_READ_REQ_LATENCY_sum"] / cyc / 256
        if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
            d["valu_lane_util"] = c["SQ_THREAD_CYCLES_VALU"] / (c["SQ_ACTIVE_INST_VALU"] * 4 * 64)
        if "SQ_BUSY_CU_CYCLES" in c:
            d["busy_cu_frac"] = c["SQ_BUSY_CU_CYCLES"] / cyc / 256
        if "SQ_ACTIVE_INST_VALU" in c:
            d["valu_active_per_simd"] = c["SQ_ACTIVE_INST_VALU"] * 4 / cyc / 1024
        if "TCC_HIT_sum" in c:
            d["l2_hit"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    out[env] = d
print(json.dumps(out, indent=1, sort_keys=True))
