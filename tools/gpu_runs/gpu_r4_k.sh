#!/bin/bash
# Round 4: kernel trace of the long-context scenario (64k prompt beside 16 decoders, 24 generated tokens) to split
# the long sequence's 44 ms TPOT into GPU kernel time vs gaps: per-kernel durations over the final decode steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4k_trace
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r4k_trace -o run --output-format csv -- python3 -m shai_amd.bench.long_context \
  --model llama31_8b --prompt-len 65536 --chunk 8192 --background 16 --gen 24 > gpurun_out/r4k_trace.log 2>&1 || { tail -20 gpurun_out/r4k_trace.log; exit 1; }
tail -1 gpurun_out/r4k_trace.log | cut -c1-300
python3 - <<'PY' > gpurun_out/r4k_summary.txt
import csv, glob, collections
f = glob.glob("gpurun_out/r4k_trace/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"][:90]
# the last 20 decode steps: find the last 20*32 decode attention launches and the window they span
da = [i for i, r in enumerate(rows) if "decode_attn_kernel" in r["Kernel_Name"]]
first = da[-20 * 32]
win = rows[first:]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
print(f"window: {len(win)} kernels, wall {(t1 - t0) / 1e6:.2f} ms, kernel busy {busy / 1e6:.2f} ms (20 decode steps)")
per = collections.defaultdict(lambda: [0, 0])
for r in win:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per[name(r)][0] += d
    per[name(r)][1] += 1
for k, (d, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:15]:
    print(f"{d / 1e6:9.2f} ms {n:6d} calls {d / n / 1e3:9.1f} us  {k}")
gaps = sorted((int(b["Start_Timestamp"]) - int(a["End_Timestamp"]), name(a), name(b)) for a, b in zip(win, win[1:]))[-8:]
for g, a, b in gaps:
    print(f"gap {g / 1e6:.2f} ms after {a} -> {b}")
PY
cat gpurun_out/r4k_summary.txt
find gpurun_out/r4k_trace -name '*kernel_trace.csv' -delete
