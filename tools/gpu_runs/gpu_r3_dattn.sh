#!/bin/bash
# Decode-attention microbenchmark per split count and context, and the decode GEMM shapes (cold weights).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_kernels.py --only dattn,decode > gpurun_out/r3d_kern.log 2>&1 || { tail -20 gpurun_out/r3d_kern.log; exit 1; }
cat gpurun_out/r3d_kern.log | tail -30
