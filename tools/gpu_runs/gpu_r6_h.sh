#!/bin/bash
# Round 6: SD2.1 batch-1 latency anatomy -- kernel table + one UNet step's dispatch sequence (durations, gaps) of
# bench.py --batch 1 (warm tuning cache, autotune off under the trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_GEMM_AUTOTUNE=0 timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r6h_sdb1 -o run -- python3 -u bench.py \
  --batch 1 --steps 2 --warmup 1 --latency-runs 0 > gpurun_out/r6h_sdb1.log 2>&1 || { tail -20 gpurun_out/r6h_sdb1.log; exit 1; }
grep '^{' gpurun_out/r6h_sdb1.log | tail -1 | cut -c1-400
python3 tools/prof_db.py $(find gpurun_out/r6h_sdb1 -name "*results.db" | head -1) --top 40 \
  --title "SD2.1 batch 1, 50 steps x 3 generates (round 6)" --seq -2500 800 > gpurun_out/r6h_sdb1.md && rm -rf gpurun_out/r6h_sdb1
head -50 gpurun_out/r6h_sdb1.md
