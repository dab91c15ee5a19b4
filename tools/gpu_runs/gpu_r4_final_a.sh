#!/bin/bash
# Round-4 closing evidence (1/2) on one MI355X: GPU suite, smoke(), the driver's default SD2.1 bench line (20 / 5).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4z_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4z_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4z_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4z_smoke.log 2>&1 || { tail -20 gpurun_out/r4z_smoke.log; exit 1; }
tail -1 gpurun_out/r4z_smoke.log | cut -c1-300
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4z_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r4z_bench_sd21.log
