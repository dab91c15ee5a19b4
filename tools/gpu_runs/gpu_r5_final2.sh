#!/bin/bash
# Round-5 last check of the final tree: GPU suite, smoke, SD2.1 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5z2_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5z2_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5z2_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z2_smoke.log 2>&1 || { tail -20 gpurun_out/r5z2_smoke.log; exit 1; }
tail -1 gpurun_out/r5z2_smoke.log | cut -c1-120
timeout -k 10 600 python -u bench.py > gpurun_out/r5z2_bench.log 2>&1 || { tail -20 gpurun_out/r5z2_bench.log; exit 1; }
grep '^{' gpurun_out/r5z2_bench.log | tail -1 | cut -c1-300
