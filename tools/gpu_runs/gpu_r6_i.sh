#!/bin/bash
# Round 6: where the SD2.1 batch-32 bench step is idle -- kernel trace of one timed step (+ warmup), the longest
# gaps between kernels, and the dispatch sequence around the end of a generate call (VAE decode, next text encode).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_GEMM_AUTOTUNE=0 timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r6i_sd -o run -- python3 -u bench.py \
  --steps 1 --warmup 1 --latency-runs 0 > gpurun_out/r6i_sd.log 2>&1 || { tail -20 gpurun_out/r6i_sd.log; exit 1; }
grep '^{' gpurun_out/r6i_sd.log | tail -1 | cut -c1-300
python3 tools/prof_db.py $(find gpurun_out/r6i_sd -name "*results.db" | head -1) --top 12 --gaps 40 \
  --title "SD2.1 batch 32, warmup + 1 timed step (round 6)" --seq -700 700 > gpurun_out/r6i_sd.md && rm -rf gpurun_out/r6i_sd
sed -n 1,70p gpurun_out/r6i_sd.md
