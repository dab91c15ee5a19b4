#!/bin/bash
# Round 5: v4 (gemm_8ph.hip) codegen A/B -- default vs VGPR-form MFMAs, plain problems + convs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab > gpurun_out/r5x_lab.log 2>&1 &&
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab_x > gpurun_out/r5x_lab_x.log 2>&1
