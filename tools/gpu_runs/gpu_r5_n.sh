#!/bin/bash
# Round 5: 16-B GLU stores (lane-quad swaps) in the ws and v4 epilogues -- GEMM tests, lab, SD2.1 bench + breakdown
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gemm_ws_gpu.py tests/test_gemm3_gpu.py tests/test_norm_handoff_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r5n_pytest.log 2>&1 || { tail -30 gpurun_out/r5n_pytest.log; exit 1; }
tail -1 gpurun_out/r5n_pytest.log
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab > gpurun_out/r5n_lab.log 2>&1 || { tail -20 gpurun_out/r5n_lab.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r5n_bench.log 2>&1 || { tail -20 gpurun_out/r5n_bench.log; exit 1; }
tail -1 gpurun_out/r5n_bench.log | cut -c1-300
timeout -k 10 300 python -u tools/op_breakdown.py --batch 32 --top 40 > gpurun_out/r5n_opbreak.log 2>&1 || { tail -20 gpurun_out/r5n_opbreak.log; exit 1; }
grep -v Warning gpurun_out/r5n_opbreak.log | head -16 | cut -c1-150
