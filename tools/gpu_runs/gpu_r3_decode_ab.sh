#!/bin/bash
# Decode A/B on one MI355X: skinny-GEMM weight stream with the nt cache policy (default) vs default policy,
# Mistral b64 bench lines + per-shape skinny bandwidth; then the long-context scenario.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for nt in 1 0; do
  SHAI_SKINNY_NT=$nt timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_mistral_nt$nt.log 2>&1 || exit $?
  echo "== mistral nt=$nt"; tail -1 gpurun_out/r3_mistral_nt$nt.log | cut -c1-420
  SHAI_SKINNY_NT=$nt SHAI_DECODE_M=64 SHAI_NUM_CFGS=0 timeout -k 10 300 python -u tools/bench_kernels.py --only decode > gpurun_out/r3_decode_nt$nt.log 2>&1 || exit $?
  grep decode_gemm gpurun_out/r3_decode_nt$nt.log
done
timeout -k 10 500 python -u -m shai_amd.bench.long_context > gpurun_out/r3_long_mixed.log 2>&1 || { tail -20 gpurun_out/r3_long_mixed.log; exit 1; }
echo "== long context (mixed)"; tail -1 gpurun_out/r3_long_mixed.log
timeout -k 10 500 python -u -m shai_amd.bench.long_context --no-mix > gpurun_out/r3_long_nomix.log 2>&1 || { tail -20 gpurun_out/r3_long_nomix.log; exit 1; }
echo "== long context (alternating)"; tail -1 gpurun_out/r3_long_nomix.log
