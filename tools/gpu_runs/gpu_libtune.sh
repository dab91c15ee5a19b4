#!/bin/bash
# hipBLASLt candidate in the GEMM autotuner: numerics, then a fresh autotune of the SD2.1 b32 bench shapes
# (tile configs vs library), then a clean bench from the saved cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" \
  > gpurun_out/pytest_lib.log 2>&1 || { tail -30 gpurun_out/pytest_lib.log; exit 1; }
tail -1 gpurun_out/pytest_lib.log
SHAI_GEMM_TUNE_FILE=none SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_lib.json timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --latency-runs 0 \
  > gpurun_out/libtune_sd21.log 2>&1 || { tail -30 gpurun_out/libtune_sd21.log; exit 1; }
echo "== tuned"; tail -1 gpurun_out/libtune_sd21.log | cut -c1-200
SHAI_GEMM_TUNE_FILE=gpurun_out/tune_lib.json timeout -k 10 600 python -u bench.py > gpurun_out/lib_sd21.log 2>&1 || exit 1
echo "== lib cache"; tail -1 gpurun_out/lib_sd21.log | cut -c1-200
timeout -k 10 600 python -u bench.py > gpurun_out/base_sd21.log 2>&1 || exit 1
echo "== committed cache"; tail -1 gpurun_out/base_sd21.log | cut -c1-200
