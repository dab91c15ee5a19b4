#!/bin/bash
# GPU check: gpu-marked tests, then the default SD2.1 bench. Each step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_sd.log 2>&1
rc=$?
tail -2 gpurun_out/bench_sd.log
exit $rc
