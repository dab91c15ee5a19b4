"""Summarise tools/gpu_runs/gpu_r3_pmc.sh output: per kernel variant, mean kernel time (kernel-trace stats) and the mean
of every collected counter over the GEMM dispatches (the skinny kernels only)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    rows = []
    for kt in sorted(glob.glob(os.path.join(root, "kt_*"))):
        cfg = kt.rsplit("_", 1)[1]
        t_us = None
        for f in glob.glob(os.path.join(kt, "**", "*kernel_stats.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "skinny" in r["Name"]:
                    t_us = float(r["AverageNs"]) / 1e3
        vals = defaultdict(list)
        for p in ("p1", "p2"):
            for f in glob.glob(os.path.join(root, f"{p}_{cfg}", "**", "*counter_collection.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if "skinny" in r.get("Kernel_Name", ""):
                        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        rows.append((cfg, t_us, {k: sum(v) / len(v) for k, v in vals.items()}))
    names = sorted({k for _, _, d in rows for k in d})
    print("| cfg | kernel us | " + " | ".join(names) + " |")
    print("|---" * (2 + len(names)) + "|")
    for cfg, t, d in rows:
        print(f"| {cfg} | {t:.1f} | " + " | ".join(f"{d.get(k, float('nan')):.4g}" for k in names) + " |")


if __name__ == "__main__":
    main(sys.argv[1])
