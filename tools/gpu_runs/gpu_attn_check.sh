#!/bin/bash
# Attention numerics, the attention microbenchmarks and the SD2.1 bench (each step time-limited).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_sd_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_attn.log 2>&1 || { tail -30 gpurun_out/pytest_attn.log; exit 1; }
tail -1 gpurun_out/pytest_attn.log
timeout -k 10 300 python -u tools/bench_kernels.py --only attn > gpurun_out/kbench_attn.log 2>&1 || exit 1
grep "^op=" gpurun_out/kbench_attn.log
timeout -k 10 600 python -u bench.py > gpurun_out/attn_sd21.log 2>&1 || exit 1
tail -1 gpurun_out/attn_sd21.log | cut -c1-200
