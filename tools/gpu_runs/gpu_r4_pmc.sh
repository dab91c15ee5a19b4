#!/bin/bash
# Round 4: PMC pass over the GEMM lab (MFMA busy / waits / LDS per kernel variant, incl. the four-wave kernel).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_SET=sq bash tools/gemm_lab/run_gpu.sh r4pmc > /dev/null || exit 1
cut -c1-300 gpurun_out/pmc_r4pmc.md
