#!/usr/bin/env python
"""Condense a tools/profile_round.sh run into profiles/<tag>_*.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied verbatim)
  profiles/<tag>_summary.json       per-kernel average duration, calls, and HBM
                                    bytes per dispatch from the FETCH_SIZE /
                                    WRITE_SIZE passes; also the per-kernel
                                    "traffic" figure bench.py --traffic reads.
PMC units (MI355X_MICROARCH.md, HBM): FETCH_SIZE and WRITE_SIZE are KiB.  The
documented gfx950 correction (FETCH_SIZE reads 1/2 of the bytes of 16-B/lane
streaming reads) applies to wide coalesced loads only; these kernels load 8 B
per lane (global_load_dwordx2 / sc1), a width the guide leaves uncalibrated, so
the raw value is reported and the x2 figure is given as an upper bound.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

KERNELS = {"backward": "cluster_kernel<1", "forward": "cluster_kernel<0"}


def main(tag, src, dst="profiles", config="c3"):
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    summary = {"tag": tag, "config": config, "kernels": {}}
    for r in rows:
        summary["kernels"][r["Name"]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                         "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6,
                                         "pct": float(r["Percentage"])}
    pmc = defaultdict(lambda: defaultdict(list))
    for name in ("fetch", "write"):
        path = os.path.join(src, name, f"{name}_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            pmc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    traffic = {}
    for key, pat in KERNELS.items():
        names = [n for n in pmc if pat in n]
        if not names:
            continue
        n = names[0]
        fetch = pmc[n].get("FETCH_SIZE", [])
        write = pmc[n].get("WRITE_SIZE", [])
        # the last dispatch of each pass is a timed step
        f, w = (fetch[-1] if fetch else 0.0) * 1024, (write[-1] if write else 0.0) * 1024
        traffic[key] = {"kernel": n, "fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes_per_launch": f + w,
                        "hbm_bytes_upper_bound": 2 * f + w, "dispatches": len(fetch)}
    summary["traffic"] = traffic
    json.dump(summary, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1)
    json.dump(traffic, open(os.path.join(dst, f"{tag}_traffic.json"), "w"), indent=1)
    for k, v in traffic.items():
        print(f"{k}: {v['kernel'][:48]} HBM {v['hbm_bytes_per_launch'] / 1e9:.3f} GB/launch "
              f"(fetch {v['fetch_bytes_raw'] / 1e9:.3f}, write {v['write_bytes'] / 1e9:.3f})")
    for n, k in sorted(summary["kernels"].items(), key=lambda kv: -kv[1]["pct"])[:6]:
        print(f"  {k['pct']:6.2f}%  {k['avg_ms']:10.3f} ms avg  x{k['calls']}  {n[:70]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:5]))
