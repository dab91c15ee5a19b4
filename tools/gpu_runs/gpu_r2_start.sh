#!/bin/bash
# Round-2 opening evidence on one MI355X: GPU test suite, SD2.1 headline bench, Mistral bench and a
# kernel-trace profile of one SD2.1 batch.  Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r2_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r2_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r2_pytest_gpu.log
timeout -k 10 500 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r2_bench_sd21.log | cut -c1-300
timeout -k 10 500 python -u bench.py --workload mistral > gpurun_out/r2_bench_mistral.log 2>&1 || exit $?
echo "== mistral"; tail -1 gpurun_out/r2_bench_mistral.log | cut -c1-300
bash tools/rocprof.sh r2_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 || exit $?
