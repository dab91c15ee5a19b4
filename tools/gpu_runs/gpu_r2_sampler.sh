#!/bin/bash
# Sampler / skinny / engine GPU tests and the Mistral b64 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_skinny_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "sampler or engine or skinny" > gpurun_out/r2s_tests.log 2>&1 || { tail -30 gpurun_out/r2s_tests.log; exit 1; }
tail -1 gpurun_out/r2s_tests.log
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r2s_bench_mistral.log 2>&1 || exit $?
echo "== mistral"; tail -1 gpurun_out/r2s_bench_mistral.log | cut -c1-700
bash tools/rocprof.sh r2s_mistral_b64 -- bench.py --workload mistral --steps 2 --warmup 1 || exit $?
grep -n "sample_kernel" gpurun_out/rocprof_r2s_mistral_b64.md
