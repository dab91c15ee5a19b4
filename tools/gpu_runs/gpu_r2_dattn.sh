#!/bin/bash
# Decode attention (packed bf16 dot products, fused RoPE + KV write) numerics, LLM engine tests, Mistral b64
# bench (fused and unfused decode) and profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_skinny_gpu.py tests/test_models_gpu.py tests/test_fp8_gpu.py \
  tests/test_mllama_gpu.py -x -q --timeout 120 --timeout-method thread -k "decode or engine or mllama or rope" \
  > gpurun_out/r2a_tests.log 2>&1 || { tail -30 gpurun_out/r2a_tests.log; exit 1; }
tail -1 gpurun_out/r2a_tests.log
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r2a_bench_mistral.log 2>&1 || exit $?
echo "== mistral fused"; tail -1 gpurun_out/r2a_bench_mistral.log | cut -c1-90; tail -1 gpurun_out/r2a_bench_mistral.log | grep -o '"p50_tpot_ms.*'
SHAI_FUSED_DECODE=0 timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r2a_bench_mistral_unfused.log 2>&1 || exit $?
echo "== mistral unfused"; tail -1 gpurun_out/r2a_bench_mistral_unfused.log | cut -c1-90; tail -1 gpurun_out/r2a_bench_mistral_unfused.log | grep -o '"p50_tpot_ms.*'
bash tools/rocprof.sh r2a_mistral_b64 -- bench.py --workload mistral --steps 2 --warmup 1 > /dev/null || exit $?
grep -n "decode_attn\|rope" gpurun_out/rocprof_r2a_mistral_b64.md
