#!/bin/bash
# Round 4: per-sequence decode split count (a long context no longer gives every short sequence 64 workgroups):
# decode / kernel tests, Mistral b64 (short contexts: no regression), then the 64k / 128k long-context lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 60; do echo "running $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_skinny_gpu.py tests/test_varlen_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r4j_pytest.log 2>&1 || { tail -30 gpurun_out/r4j_pytest.log; exit 1; }
tail -1 gpurun_out/r4j_pytest.log
timeout -k 10 300 python -u bench.py --workload mistral --steps 2 --warmup 1 > gpurun_out/r4j_mistral.log 2>&1 || exit $?
echo "mistral: $(tail -1 gpurun_out/r4j_mistral.log | cut -c1-200)"
for P in 65536 127744; do
  timeout -k 10 400 python -u -m shai_amd.bench.long_context --model llama31_8b --prompt-len $P --chunk 8192 \
    --background 16 --gen 128 > gpurun_out/r4j_long_$P.log 2>&1 || { tail -20 gpurun_out/r4j_long_$P.log; exit 1; }
  tail -1 gpurun_out/r4j_long_$P.log
done
