#!/bin/bash
# Round 5: PMC (SQ set) over the W-stationary lab problems.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_SET=sq bash tools/gemm_lab/run_gpu.sh r5d --ws > /dev/null 2>&1 || { tail -20 gpurun_out/pmc_r5d.log; exit 1; }
grep -E "ws_kernel|gemm4_kernel<0, (false|true), (0|2), false, 20, 320>" gpurun_out/pmc_r5d.md
