#!/usr/bin/env python3
"""Aggregate a rocprofv3 --pmc counter_collection.csv per (kernel, grid) for the GEMM lab.

Prints one row per kernel instantiation and grid size with the mean of each counter over dispatches,
plus derived ratios: MFMA busy share of busy cycles and the wait shares of wave cycles.
"""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void shai::", "").split("(")[0]
    return name[:60]


def main(path: str) -> None:
    acc = defaultdict(lambda: defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            k = (short(r.get("Kernel_Name", "?")), r.get("Grid_Size", r.get("Grid_Size_X", "?")))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted({c for v in acc.values() for c in v})
    print("| kernel | grid | " + " | ".join(names) + " | mfma/busy | wait_any/wave | wait_inst/wave |")
    print("|---|---|" + "---|" * (len(names) + 3))
    for (kn, grid), cs in sorted(acc.items()):
        mean = {c: sum(v) / len(v) for c, v in cs.items()}
        busy = mean.get("SQ_BUSY_CYCLES", 0.0)
        wave = mean.get("SQ_WAVE_CYCLES", 0.0)
        mf = mean.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        row = [f"{mean.get(c, 0.0):.3g}" for c in names]
        r1 = f"{mf / busy:.3f}" if busy else "-"
        r2 = f"{mean.get('SQ_WAIT_ANY', 0.0) / wave:.3f}" if wave else "-"
        r3 = f"{mean.get('SQ_WAIT_INST_ANY', 0.0) / wave:.3f}" if wave else "-"
        print(f"| {kn} | {grid} | " + " | ".join(row) + f" | {r1} | {r2} | {r3} |")


if __name__ == "__main__":
    main(sys.argv[1])
