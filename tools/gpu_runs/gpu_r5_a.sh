#!/bin/bash
# Round 5, first GPU call: fresh per-op breakdown of one SD2.1 UNet step (b32 CFG), the low-K GEMM table,
# the GEMM lab over the SD2.1 shapes (baseline for the new kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/op_breakdown.py --batch 32 --top 70 > gpurun_out/r5a_opbreak.log 2>&1 || { tail -30 gpurun_out/r5a_opbreak.log; exit 1; }
head -40 gpurun_out/r5a_opbreak.log | cut -c1-200
timeout -k 10 200 python -u tools/bench_sd_lowk.py > gpurun_out/r5a_lowk.log 2>&1 || { tail -30 gpurun_out/r5a_lowk.log; exit 1; }
cat gpurun_out/r5a_lowk.log
timeout -k 10 400 ./tools/gemm_lab/bin/gemm_lab full > gpurun_out/r5a_lab.log 2>&1 || { tail -30 gpurun_out/r5a_lab.log; exit 1; }
grep -c MISMATCH gpurun_out/r5a_lab.log
