#!/bin/bash
# New GPU tests of this session's engine changes, then the big-LLM lines: Llama-3-8B (128k vocab) b64 and
# DeepSeek-R1-Distill-Llama-70B bf16 (random init, ONE GPU) at batch 1 and 16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_skinny_gpu.py tests/test_varlen_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r3_newtests.log 2>&1 || { tail -40 gpurun_out/r3_newtests.log; exit 1; }
tail -1 gpurun_out/r3_newtests.log
timeout -k 10 400 python -u bench.py --workload mistral --llm-model llama3_8b > gpurun_out/r3_llama3_8b.log 2>&1 || { tail -20 gpurun_out/r3_llama3_8b.log; exit 1; }
echo "== llama3-8b b64"; tail -1 gpurun_out/r3_llama3_8b.log
for b in 1 16; do
  timeout -k 10 500 python -u bench.py --workload mistral --llm-model deepseek_r1_distill_70b --batch $b --gen-len 64 --steps 2 --warmup 1 \
    > gpurun_out/r3_ds70b_b$b.log 2>&1 || { tail -20 gpurun_out/r3_ds70b_b$b.log; exit 1; }
  echo "== deepseek-70b b$b"; tail -1 gpurun_out/r3_ds70b_b$b.log
done
