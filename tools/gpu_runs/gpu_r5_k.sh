#!/bin/bash
# Round 5: decode GEMM rate vs M (X-operand traffic probe)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_DECODE_M=1,16,32,48,64 timeout -k 10 500 python -u tools/bench_kernels.py --only decode > gpurun_out/r5k_decode.log 2>&1 || { tail -20 gpurun_out/r5k_decode.log; exit 1; }
grep decode_gemm gpurun_out/r5k_decode.log | cut -c1-300
