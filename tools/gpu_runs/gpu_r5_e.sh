#!/bin/bash
# Round 5: W-stationary kernel ablations (no stores / no MFMA / no DMA / DMA only) to price each component.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab --ws > gpurun_out/r5e_lab.log 2>&1 || { cat gpurun_out/r5e_lab.log; exit 1; }
grep -E "==|v4_320w |ws_" gpurun_out/r5e_lab.log | grep -v "OK$"
grep -c MISMATCH gpurun_out/r5e_lab.log || true
