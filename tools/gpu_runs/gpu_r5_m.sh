#!/bin/bash
# Round 5: W-stationary GEMM lab (K = 320 problems + ablations) after the activation rewrite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab --ws > gpurun_out/r5m_lab.log 2>&1
