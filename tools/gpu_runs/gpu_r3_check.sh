#!/bin/bash
# Round-3 check on one MI355X: GPU test suite, then the Mistral decode bench with the acq_rel split-K
# ticket (default) and the relaxed one (A/B of the release/acquire cost).  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3_pytest_gpu.log
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r3_mistral_acqrel.log 2>&1 || exit $?
echo "== mistral acq_rel"; tail -1 gpurun_out/r3_mistral_acqrel.log | cut -c1-600
SHAI_SK_RELAXED_TICKET=1 timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r3_mistral_relaxed.log 2>&1 || exit $?
echo "== mistral relaxed"; tail -1 gpurun_out/r3_mistral_relaxed.log | cut -c1-600
timeout -k 10 400 python -u -m shai_amd.bench.long_context > gpurun_out/r3_long_mixed.log 2>&1 || { tail -20 gpurun_out/r3_long_mixed.log; exit 1; }
echo "== long context (mixed)"; tail -1 gpurun_out/r3_long_mixed.log
timeout -k 10 400 python -u -m shai_amd.bench.long_context --no-mix > gpurun_out/r3_long_nomix.log 2>&1 || { tail -20 gpurun_out/r3_long_nomix.log; exit 1; }
echo "== long context (alternating)"; tail -1 gpurun_out/r3_long_nomix.log
