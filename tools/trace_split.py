#!/usr/bin/env python3
"""tools/trace_split.py DIR SPEC... — per-spec mean kernel durations from a rocprofv3 --kernel-trace
of tools/sweep_part.py (each spec makes 7 probe_partitioned calls: 2 warm-up + 5 timed)."""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
specs = sys.argv[2:]
seq = defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    for key in ("slot_split", "probe_win", "probe_pair"):
        if key in n:
            seq[key if key == "slot_split" else "probe"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for i, sp in enumerate(specs):
    sl = seq["slot_split"][7 * i + 2:7 * i + 7]
    pr = seq["probe"][7 * i + 2:7 * i + 7]
    print(f"{sp:24s} split {sum(sl) / max(len(sl), 1):7.3f} ms  probe {sum(pr) / max(len(pr), 1):7.3f} ms")
