#!/bin/bash
# Round 6: flash128x2 (D = 128, two query groups per wave) -- attention / varlen / Flux / mllama GPU tests, then the
# A/B against flash2<128> at the Flux / prefill shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_varlen_gpu.py -k "flash or attn or varlen" -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r6d_attn_tests.log 2>&1 || { tail -40 gpurun_out/r6d_attn_tests.log; exit 1; }
tail -1 gpurun_out/r6d_attn_tests.log
timeout -k 10 300 python -u tools/bench_attn128.py gpurun_out/r6d_attn128.json > gpurun_out/r6d_attn128.log 2>&1 \
  || { tail -20 gpurun_out/r6d_attn128.log; exit 1; }
cat gpurun_out/r6d_attn128.log | grep '^{'
timeout -k 10 600 python -u -m pytest tests/test_flux_gpu.py tests/test_mllama_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r6d_flux_tests.log 2>&1 || { tail -40 gpurun_out/r6d_flux_tests.log; exit 1; }
tail -1 gpurun_out/r6d_flux_tests.log
timeout -k 10 600 python -u bench.py --workload flux --height 1024 --width 1024 --steps 2 --warmup 1 --inference-steps 10 \
  > gpurun_out/r6d_flux1024.log 2>&1 || { tail -20 gpurun_out/r6d_flux1024.log; exit 1; }
grep '^{' gpurun_out/r6d_flux1024.log | tail -1 | cut -c1-400
