#!/usr/bin/env python3
"""Summarise a rocprofv3 SQLite database (``rocprofv3 --kernel-trace -d DIR -o NAME`` writes ``DIR/NAME_results.db``
on ROCm 7.x) as a markdown kernel table: total time, calls, mean, share, plus the busy fraction of the trace (kernel
time over the span from the first kernel start to the last kernel end, i.e. what launch gaps cost).

    python tools/prof_db.py gpurun_out/prof/run_results.db [--top 30] [--title "..."] [--skip-ms 0]

``--skip-ms`` drops kernels that start within that many ms of the first one (warm-up / autotune phase).
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--title", default=None)
    ap.add_argument("--skip-ms", type=float, default=0.0)
    ap.add_argument("--seq", type=int, nargs=2, default=None, metavar=("START", "N"),
                    help="also list N dispatches in launch order from index START (negative: from the end), "
                         "with each one's duration and the gap before it")
    ap.add_argument("--gaps", type=int, default=0, metavar="N",
                    help="also list the N longest idle gaps between consecutive kernels (and the gap total)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, duration from kernels order by start").fetchall()
    if not rows:
        print("no kernels in", a.db)
        return
    t0 = rows[0][1] + a.skip_ms * 1e6
    rows = [r for r in rows if r[1] >= t0]
    agg = {}
    for name, start, dur in rows:
        e = agg.setdefault(name, [0, 0])
        e[0] += 1
        e[1] += dur
    total = sum(v[1] for v in agg.values())
    span = max(r[1] + r[2] for r in rows) - rows[0][1]
    print(f"### {a.title or a.db}\n")
    print(f"Kernel time {total / 1e6:.2f} ms over a {span / 1e6:.2f} ms span ({100 * total / max(span, 1):.1f} % busy), "
          f"{len(rows)} dispatches.\n")
    print("| ms | calls | % | avg us | kernel |")
    print("|---:|---:|---:|---:|---|")
    for name, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        nm = name if len(name) <= 110 else name[:107] + "..."
        print(f"| {d / 1e6:.2f} | {n} | {100 * d / total:.1f} | {d / n / 1e3:.1f} | `{nm}` |")
    if a.gaps:
        gl = []
        end = rows[0][1] + rows[0][2]
        for i in range(1, len(rows)):
            g = rows[i][1] - end
            if g > 0:
                gl.append((g, i))
            end = max(end, rows[i][1] + rows[i][2])
        tot = sum(g for g, _ in gl)
        big = sum(g for g, _ in gl if g > 50e3)
        print(f"\n#### idle gaps: {tot / 1e6:.2f} ms in all, {big / 1e6:.2f} ms in gaps over 50 us\n")
        print("| gap us | at dispatch | after | before |")
        print("|---:|---:|---|---|")
        for g, i in sorted(gl, reverse=True)[:a.gaps]:
            print(f"| {g / 1e3:.1f} | {i} | `{rows[i - 1][0][:60]}` | `{rows[i][0][:60]}` |")
    if a.seq:
        st, n = a.seq
        st = st if st >= 0 else len(rows) + st
        seq = rows[st:st + n]
        busy = sum(r[2] for r in seq)
        span = seq[-1][1] + seq[-1][2] - seq[0][1] if seq else 0
        print(f"\n#### dispatches {st}..{st + len(seq) - 1} in launch order: {busy / 1e3:.1f} us of kernels over a "
              f"{span / 1e3:.1f} us span\n")
        print("| # | us | gap us | kernel |")
        print("|---:|---:|---:|---|")
        prev_end = None
        for i, (name, start, dur) in enumerate(seq):
            gap = (start - prev_end) / 1e3 if prev_end is not None else 0.0
            prev_end = start + dur
            nm = name if len(name) <= 100 else name[:97] + "..."
            print(f"| {st + i} | {dur / 1e3:.1f} | {gap:.1f} | `{nm}` |")


if __name__ == "__main__":
    main()
