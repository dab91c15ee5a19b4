#!/bin/bash
# Round 5: LDS-staged GLU stores in the W-stationary kernel -- lab (numerics + timing), ws tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab --ws > gpurun_out/r5t_lab.log 2>&1 || { tail -20 gpurun_out/r5t_lab.log; exit 1; }
grep -A8 "glu" gpurun_out/r5t_lab.log | grep -E "==|ws_|MISM" | head -24
timeout -k 10 400 python -u -m pytest tests/test_gemm_ws_gpu.py tests/test_norm_handoff_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r5t_pytest.log 2>&1 || { tail -30 gpurun_out/r5t_pytest.log; exit 1; }
tail -1 gpurun_out/r5t_pytest.log
