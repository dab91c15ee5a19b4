#!/bin/bash
# Round 4: long-context lines at the reference's configured length (max_model_len 128000,
# cova/mllama-32-11b-vllm-trn1-config.yaml:12-16): Llama-3.1-8B (128k RoPE), a 64k and a ~128k prompt prefilled in
# 8k packed chunks beside 16 decoding sequences, then decoded (TTFT, TPOT); first a batch-1 SD2.1 profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 60; do echo "long-context running $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
# batch-1 SD2.1 kernel profile (single-request latency, verdict item: p50 <= 300 ms)
bash tools/rocprof.sh r4g_sd21_bs1 -- bench.py --batch 1 --steps 3 --warmup 1 --latency-runs 0 || exit $?
for P in 65536 127744; do
  timeout -k 10 500 python -u -m shai_amd.bench.long_context --model llama31_8b --prompt-len $P --chunk 8192 \
    --background 16 --gen 128 > gpurun_out/r4g_long_$P.log 2>&1 || { tail -20 gpurun_out/r4g_long_$P.log; exit 1; }
  tail -1 gpurun_out/r4g_long_$P.log
done
