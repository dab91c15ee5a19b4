#!/bin/bash
# Split-K fold change: GEMM / skinny numerics, Mistral b64 bench and profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_skinny_gpu.py tests/test_gemm3_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "skinny or gemm or split" > gpurun_out/r2k_tests.log 2>&1 || { tail -30 gpurun_out/r2k_tests.log; exit 1; }
tail -1 gpurun_out/r2k_tests.log
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r2k_bench_mistral.log 2>&1 || exit $?
echo "== mistral"; tail -1 gpurun_out/r2k_bench_mistral.log | cut -c1-90; tail -1 gpurun_out/r2k_bench_mistral.log | grep -o '"p50_tpot_ms.*'
bash tools/rocprof.sh r2k_mistral_b64 -- bench.py --workload mistral --steps 2 --warmup 1 > /dev/null || exit $?
grep -n "splitk\|decode_attn" gpurun_out/rocprof_r2k_mistral_b64.md
