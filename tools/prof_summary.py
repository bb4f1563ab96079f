#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_TAG) into profiles/:

  profiles/TAG_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as written by rocprofv3)
  profiles/TAG_pmc.json           per-kernel PMC counters (last dispatch of each counter pass)
  profiles/pmc_<workload>.json    HBM traffic per probe launch for bench.py's roofline.traffic

Traffic = (FETCH_SIZE + WRITE_SIZE) * 1024 bytes per launch (rocprofv3 reports both in KiB).  The
gfx950 x2 correction of FETCH_SIZE (MI355X_MICROARCH.md §HBM) applies to wide coalesced streaming
reads; the probe's reads are dominated by random 32-byte window gathers issued as 64-byte requests
(FETCH_SIZE == TCC_EA0_RDREQ x 64 B, RDREQ_32B == 0), so no factor is applied — both raw numbers are
kept in TAG_pmc.json.
  usage: tools/prof_summary.py TAG [--n-probe N --n-build N]
"""
import argparse
import collections
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="probe_chunks")
    ap.add_argument("--n-probe", type=int, default=1 << 30)
    ap.add_argument("--n-build", type=int, default=1 << 26)
    ap.add_argument("--workload", default="c2", help="writes profiles/pmc_<workload>.json for bench.py")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(dst, f"{a.tag}_kernel_stats.csv"))
    stats = {}
    with open(os.path.join(src, "kt", "kt_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    pmc = collections.defaultdict(dict)
    for d in sorted(os.listdir(src)):
        p = os.path.join(src, d, "pmc_counter_collection.csv")
        if not d.startswith("pmc_") or not os.path.exists(p):
            continue
        with open(p) as f:
            for r in csv.DictReader(f):
                pmc[r["Kernel_Name"]][r["Counter_Name"]] = float(r["Counter_Value"])
                pmc[r["Kernel_Name"]]["VGPR_Count"] = int(r["VGPR_Count"])
    out = {"tag": a.tag, "kernel_stats": stats, "pmc": pmc}
    k = pmc.get(a.kernel, {})
    if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
        fetch, write = k["FETCH_SIZE"] * 1024, k["WRITE_SIZE"] * 1024
        traffic = fetch + write
        avg_ns = stats.get(a.kernel, {}).get("avg_ns")
        out["traffic"] = {"fetch_bytes": fetch, "write_bytes": write, "hbm_bytes_per_launch": traffic,
                          "bytes_per_probe_tuple": traffic / a.n_probe,
                          "rdreq_per_tuple": k.get("TCC_EA0_RDREQ_sum", 0) / a.n_probe,
                          "l2_hit_rate": (k["TCC_HIT_sum"] / (k["TCC_HIT_sum"] + k["TCC_MISS_sum"])
                                          if "TCC_HIT_sum" in k else None),
                          "hbm_GBps": traffic / avg_ns if avg_ns else None}
        with open(os.path.join(dst, f"pmc_{a.workload}.json"), "w") as f:
            json.dump({"tag": a.tag, "kernel": a.kernel, "n_probe": a.n_probe, "n_build": a.n_build,
                       "hbm_bytes_per_launch": traffic, "fetch_size_kib": k["FETCH_SIZE"],
                       "write_size_kib": k["WRITE_SIZE"], "kernel_avg_ns": avg_ns}, f, indent=1)
    with open(os.path.join(dst, f"{a.tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out.get("traffic", {}), indent=1))


if __name__ == "__main__":
    main()
