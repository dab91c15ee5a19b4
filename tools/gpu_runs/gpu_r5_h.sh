#!/bin/bash
# flash64 variants A/B in the attention lab (default codegen, then attn_lab_x if built)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 180 ./tools/gemm_lab/bin/attn_lab > gpurun_out/r5h_attn.log 2>&1 &&
if [ -x tools/gemm_lab/bin/attn_lab_x ]; then timeout -k 10 180 ./tools/gemm_lab/bin/attn_lab_x > gpurun_out/r5h_attn_x.log 2>&1; fi
