"""Summarise rocprofv3 csv output under gpurun_out/prof_TAG (kernel stats + PMC)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(tag):
    root = f"gpurun_out/prof_{tag}"
    out = {}
    for f in glob.glob(f"{root}/kt/**/*kernel_stats.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        for r in rows:
            print(f"{r['Name'][:60]:60s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs'])/1e6:9.3f} "
                  f"total_ms={float(r['TotalDurationNs'])/1e6:9.2f} pct={float(r['Percentage']):6.2f}")
        out["stats"] = rows
    for f in glob.glob(f"{root}/pmc_*/**/*counter_collection.csv", recursive=True):
        acc = defaultdict(lambda: defaultdict(float))
        n = defaultdict(set)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "enhance" not in k:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
        for k, d in acc.items():
            print(k[:50], "dispatches", len(n[k]))
            for c, v in sorted(d.items()):
                print(f"   {c:28s} {v / max(1, len(n[k])):.4g}")
        out.setdefault("pmc", {})[f] = {k: dict(v) for k, v in acc.items()}
    json.dump(out, open(f"{root}/summary.json", "w"), indent=1, default=str)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "dev")
