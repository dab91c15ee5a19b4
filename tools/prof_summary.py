#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into a markdown table."""
import csv
import sys


def main(d, top=30, title=None):
    rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"### {title or d}", "", f"Total kernel time: {tot / 1e6:.2f} ms", "",
           "| ms | calls | % | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 100:
            name = name[:100] + "..."
        out.append(f"| {float(r['TotalDurationNs']) / 1e6:.2f} | {r['Calls']} | {float(r['Percentage']):.1f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | `{name}` |")
    return "\n".join(out)


if __name__ == "__main__":
    print(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30, sys.argv[3] if len(sys.argv) > 3 else None))
