#!/bin/bash
# W8A8 fp8 MFMA GEMM: numerics, then TF/s against the bf16 GEMM on prefill shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fp8_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3_f8_tests.log 2>&1 || { tail -40 gpurun_out/r3_f8_tests.log; exit 1; }
tail -1 gpurun_out/r3_f8_tests.log
timeout -k 10 300 python -u tools/bench_kernels.py --only f8 > gpurun_out/r3_f8_bench.log 2>&1 || { tail -20 gpurun_out/r3_f8_bench.log; exit 1; }
grep "op=" gpurun_out/r3_f8_bench.log
