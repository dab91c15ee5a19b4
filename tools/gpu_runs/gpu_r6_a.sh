#!/bin/bash
# Round 6 first box: the changed contracts (gemm_ws / tile activation rejection, TP overlap default slabs + generic
# slab loop) and a 1-GPU SD2.1 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_ws_gpu.py tests/test_p2p_gpu.py tests/test_gemm3_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6a_pytest.log 2>&1 || { tail -40 gpurun_out/r6a_pytest.log; exit 1; }
tail -2 gpurun_out/r6a_pytest.log
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6a_bench.log 2>&1 || { tail -20 gpurun_out/r6a_bench.log; exit 1; }
grep '^{' gpurun_out/r6a_bench.log | tail -1 | cut -c1-500
