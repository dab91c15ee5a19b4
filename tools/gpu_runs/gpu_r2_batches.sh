#!/bin/bash
# Mistral-7B decode throughput at larger continuous-batching caps and with fp8 weights (README table).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "b128:--batch 128" "b256:--batch 256" "fp8:--quantization fp8"; do
  n=${spec%%:*}; args=${spec#*:}
  timeout -k 10 400 python -u bench.py --workload mistral $args > gpurun_out/r2b_$n.log 2>&1 || exit $?
  echo "== $n"; tail -1 gpurun_out/r2b_$n.log | cut -c1-100; tail -1 gpurun_out/r2b_$n.log | grep -o '"p50_ttft_ms.*'
done
