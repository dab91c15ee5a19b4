#!/bin/bash
# Round-3 re-entry check on one MI355X (freshly rebuilt libraries): GPU test suite, smoke(), the driver's
# default SD2.1 bench line, the Mistral line, then a kernel profile of one SD2.1 batch.  Each GPU step
# has its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3e_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3e_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3e_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3e_smoke.log 2>&1 || { tail -20 gpurun_out/r3e_smoke.log; exit 1; }
tail -1 gpurun_out/r3e_smoke.log | cut -c1-300
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3e_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r3e_bench_sd21.log | cut -c1-400
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r3e_bench_mistral.log 2>&1 || exit $?
echo "== mistral"; tail -1 gpurun_out/r3e_bench_mistral.log | cut -c1-400
bash tools/rocprof.sh r3e_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0
