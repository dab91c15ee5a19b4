#!/bin/bash
# Round 5: W-stationary kernel, AGPR-resident weights + previous tile's epilogue interleaved with this tile's MFMAs:
# lab timing + its forced numerics tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab --ws > gpurun_out/r5c_lab.log 2>&1 || { cat gpurun_out/r5c_lab.log; exit 1; }
grep -E "==|v4_320w |ws_320|MISMATCH" gpurun_out/r5c_lab.log | grep -v "OK$"
grep -c MISMATCH gpurun_out/r5c_lab.log || true
timeout -k 10 300 python -u -m pytest tests/test_gemm_ws_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5c_pytest.log 2>&1 || { tail -30 gpurun_out/r5c_pytest.log; exit 1; }
tail -2 gpurun_out/r5c_pytest.log
