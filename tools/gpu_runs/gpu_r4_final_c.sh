#!/bin/bash
# Round-4 closing check on the final tree: GPU suite, smoke, Mistral b64, the 128k long-context line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4zc_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4zc_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4zc_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4zc_smoke.log 2>&1 || { tail -20 gpurun_out/r4zc_smoke.log; exit 1; }
tail -1 gpurun_out/r4zc_smoke.log | cut -c1-200
timeout -k 10 300 python -u bench.py --workload mistral --steps 2 --warmup 1 > gpurun_out/r4zc_mistral.log 2>&1 || exit $?
echo "mistral: $(tail -1 gpurun_out/r4zc_mistral.log | cut -c1-120)"
timeout -k 10 400 python -u -m shai_amd.bench.long_context --model llama31_8b --prompt-len 127744 --chunk 8192 \
  --background 16 --gen 128 > gpurun_out/r4zc_long.log 2>&1 || { tail -20 gpurun_out/r4zc_long.log; exit 1; }
tail -1 gpurun_out/r4zc_long.log | cut -c1-420
