#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats output directory into a markdown table.

Accepts the CSV layout (``--output-format csv``: run_kernel_stats.csv) or the
default rocpd SQLite database (``*_results.db``)."""
import csv
import glob
import os
import sqlite3
import sys


def _rows(d):
    """-> list of (name, calls, total_ns, avg_ns)."""
    p = os.path.join(d, "run_kernel_stats.csv")
    if os.path.exists(p):
        return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]))
                for r in csv.DictReader(open(p))]
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not dbs:
        raise SystemExit(f"no run_kernel_stats.csv or *.db under {d}")
    out = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, n, tot in c.execute("select name, count(*), sum(duration) from kernels group by name"):
            a = out.setdefault(name, [0, 0.0])
            a[0] += n
            a[1] += float(tot)
    return [(k, v[0], v[1], v[1] / max(1, v[0])) for k, v in out.items()]


def main(d, top=30, title=None):
    rows = _rows(d)
    tot = sum(r[2] for r in rows)
    out = [f"### {title or d}", "", f"Total kernel time: {tot / 1e6:.2f} ms", "",
           "| ms | calls | % | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for name, calls, t, avg in sorted(rows, key=lambda r: -r[2])[:top]:
        name = name.replace("|", "/")
        if len(name) > 100:
            name = name[:100] + "..."
        out.append(f"| {t / 1e6:.2f} | {calls} | {100 * t / tot:.1f} | {avg / 1e3:.1f} | `{name}` |")
    return "\n".join(out)


if __name__ == "__main__":
    print(main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30, sys.argv[3] if len(sys.argv) > 3 else None))
