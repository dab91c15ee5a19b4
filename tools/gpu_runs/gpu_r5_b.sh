#!/bin/bash
# Round 5: W-stationary low-K GEMM (gemm_ws.hip) in the lab against v4 / w4 on the K = 320 shapes; the P2P / TP
# tests touched this round (slab-staged reduce, fused + overlapped row-parallel stage), the forced-config GEMM tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab --ws > gpurun_out/r5b_lab.log 2>&1 || { cat gpurun_out/r5b_lab.log; exit 1; }
grep -v "^  .*OK$" gpurun_out/r5b_lab.log
timeout -k 10 600 python -u -m pytest tests/test_gemm_ws_gpu.py tests/test_p2p_gpu.py tests/test_gemm3_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r5b_pytest.log 2>&1 || { tail -40 gpurun_out/r5b_pytest.log; exit 1; }
tail -3 gpurun_out/r5b_pytest.log
