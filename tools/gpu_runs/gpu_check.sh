#!/bin/bash
# Full GPU test suite, then the given bench workloads (default: sd21 + mistral).  Each step has its own
# time limit; the script stops at the first failing step.
#   bash tools/gpu_runs/gpu_check.sh [workload ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
[ $# -gt 0 ] || set -- sd21 mistral
for wl in "$@"; do
  timeout -k 10 900 python -u bench.py --workload $wl > gpurun_out/bench_$wl.log 2>&1
  rc=$?
  echo "== $wl rc=$rc"; tail -1 gpurun_out/bench_$wl.log | cut -c1-600
  [ $rc -eq 0 ] || exit $rc
done
