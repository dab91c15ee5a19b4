#!/bin/bash
# Full GPU test suite, Mistral-7B b64 bench and its kernel-trace profile.  Each GPU step has its own time
# limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r2c_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r2c_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r2c_pytest_gpu.log
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r2c_bench_mistral.log 2>&1 || exit $?
echo "== mistral"; tail -1 gpurun_out/r2c_bench_mistral.log | cut -c1-700
bash tools/rocprof.sh r2c_mistral_b64 -- bench.py --workload mistral --steps 2 --warmup 1 || exit $?
