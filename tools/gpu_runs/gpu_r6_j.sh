#!/bin/bash
# Round 6: is the v4 3x3 conv (SD2.1 320 / 640-level, batch-64 shape) bound by the LDS array or by the matrix pipe?
# SQ PMC pass (one pass each, 8 SQ + 2 GRBM counters at most).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lvl in 320 640; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE \
    SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
    -d gpurun_out/r6j_$lvl -o run --output-format csv -- python3 tools/pmc_conv.py $lvl > gpurun_out/r6j_$lvl.log 2>&1 \
    || { tail -5 gpurun_out/r6j_$lvl.log; exit 1; }
  f=$(find gpurun_out/r6j_$lvl -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$lvl" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    if "gemm" not in k and "conv" not in k:
        continue
    n = max(cnt[(k, "GRBM_GUI_ACTIVE")], 1)
    gui = d["GRBM_GUI_ACTIVE"]
    print(sys.argv[2], k, "dispatches", n)
    print("  MFMA util (busy / (gui x 4 SIMD x 256 CU / 8 XCD...)): mfma_busy/gui =", round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / gui, 3))
    print("  LDS_IDX_ACTIVE / BUSY_CYCLES =", round(d["SQ_LDS_IDX_ACTIVE"] / max(d["SQ_BUSY_CYCLES"], 1), 3),
          " LDS_IDX_ACTIVE / gui =", round(d["SQ_LDS_IDX_ACTIVE"] / gui, 3))
    print("  bank conflict / LDS active =", round(d["SQ_LDS_BANK_CONFLICT"] / max(d["SQ_LDS_IDX_ACTIVE"], 1), 3),
          " wait_inst_lds / wave_cycles =", round(d["SQ_WAIT_INST_LDS"] / max(d["SQ_WAVE_CYCLES"], 1), 3),
          " wait_any / wave_cycles =", round(d["SQ_WAIT_ANY"] / max(d["SQ_WAVE_CYCLES"], 1), 3))
    print("  raw:", {c: int(v) for c, v in d.items()})
PY
  rm -rf gpurun_out/r6j_$lvl
done
