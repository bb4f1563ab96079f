#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_TAG) into profiles/:

  profiles/TAG_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as written by rocprofv3)
  profiles/TAG_pmc.json           per-kernel PMC counters (last dispatch of each counter pass)
  profiles/pmc_<workload>_<path>.json  HBM traffic per step (summed over the step's kernels) for
                                  bench.py's roofline.traffic

Traffic = HBM bytes per launch from the L2's memory-side request counters, by request size:
  reads  = 128 B x TCC_EA0_RDREQ_128B + 64 B x TCC_EA0_RDREQ_64B + 32 B x TCC_EA0_RDREQ_32B
  writes = 64 B x TCC_EA0_WRREQ_64B + 32 B x (TCC_EA0_WRREQ - TCC_EA0_WRREQ_64B)
Every read miss of the probe is a whole 128-B line (RDREQ_128B == RDREQ), which FETCH_SIZE tallies at
64 B (MI355X_MICROARCH.md §HBM: double it) — so the request-size form equals 2 x FETCH_SIZE here.  The
raw FETCH_SIZE / WRITE_SIZE (KiB) are kept in TAG_pmc.json beside it.
  usage: tools/prof_summary.py TAG [--kernel a,b] [--path partitioned] [--n-probe N --n-build N]
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
    ap.add_argument("--kernel", default="probe_chunks",
                    help="kernel name(s) making up one step, comma-separated (their traffic is summed)")
    ap.add_argument("--path", default="chunk", help="bench.py --path the profile belongs to")
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
    hp = os.path.join(src, "build_hash.txt")  # tools/profile.sh: ccj_build_hash of the profiled library
    csrc_hash = open(hp).read().strip() if os.path.exists(hp) else None
    out = {"tag": a.tag, "csrc_hash": csrc_hash, "kernel_stats": stats, "pmc": pmc}
    names = a.kernel.split(",")
    per = {}
    for name in names:
        k = pmc.get(name, {})
        if "TCC_EA0_RDREQ_128B_sum" not in k or "TCC_EA0_WRREQ_sum" not in k:
            per = None
            break
        fetch = (128 * k["TCC_EA0_RDREQ_128B_sum"] + 64 * k.get("TCC_EA0_RDREQ_64B_sum", 0)
                 + 32 * k.get("TCC_EA0_RDREQ_32B_sum", 0))
        w64 = k.get("TCC_EA0_WRREQ_64B_sum", k["TCC_EA0_WRREQ_sum"])
        write = 64 * w64 + 32 * (k["TCC_EA0_WRREQ_sum"] - w64)
        per[name] = {"fetch_bytes": fetch, "write_bytes": write, "hbm_bytes": fetch + write,
                     "rdreq_per_tuple": k.get("TCC_EA0_RDREQ_sum", 0) / a.n_probe,
                     "l2_req_per_tuple": k.get("TCC_REQ_sum", 0) / a.n_probe if "TCC_REQ_sum" in k else None,
                     "l2_hit_rate": (k["TCC_HIT_sum"] / (k["TCC_HIT_sum"] + k["TCC_MISS_sum"])
                                     if "TCC_HIT_sum" in k else None),
                     "avg_ns": stats.get(name, {}).get("avg_ns"),
                     "fetch_size_kib": k.get("FETCH_SIZE"), "write_size_kib": k.get("WRITE_SIZE")}
    if per:
        traffic = sum(v["hbm_bytes"] for v in per.values())
        ns = [v["avg_ns"] for v in per.values()]
        avg_ns = sum(ns) if all(ns) else None
        out["traffic"] = {"kernels": per, "hbm_bytes_per_launch": traffic,
                          "bytes_per_probe_tuple": traffic / a.n_probe,
                          "hbm_GBps": traffic / avg_ns if avg_ns else None}
        with open(os.path.join(dst, f"pmc_{a.workload}_{a.path}.json"), "w") as f:
            json.dump({"tag": a.tag, "csrc_hash": csrc_hash, "kernels": names, "n_probe": a.n_probe, "n_build": a.n_build,
                       "hbm_bytes_per_launch": traffic, "kernels_ms": {n: v["avg_ns"] / 1e6 if v["avg_ns"] else None
                                                                    for n, v in per.items()},
                       "per_kernel": per, "kernels_avg_ns_sum": avg_ns}, f, indent=1)
    with open(os.path.join(dst, f"{a.tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out.get("traffic", {}), indent=1))


if __name__ == "__main__":
    main()
