#!/bin/bash
# Extra round-3 bench lines: T5-v1.1-large embeddings (caption 128 / prompt 32 tokens: the reference publishes
# 0.20 s / 0.09 s single-request latency on inf2) and Flux.1-dev at 1024^2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in 128 32; do
  timeout -k 10 400 python -u bench.py --workload t5 --prompt-len $L --steps 10 --warmup 2 > gpurun_out/r3m_t5_$L.log 2>&1 || { tail -20 gpurun_out/r3m_t5_$L.log; exit 1; }
  echo "== t5 $L"; tail -1 gpurun_out/r3m_t5_$L.log
done
timeout -k 10 600 python -u bench.py --workload flux --height 1024 --width 1024 --steps 2 --warmup 1 --latency-runs 1 \
  > gpurun_out/r3m_flux1024.log 2>&1 || { tail -20 gpurun_out/r3m_flux1024.log; exit 1; }
echo "== flux 1024"; tail -1 gpurun_out/r3m_flux1024.log
