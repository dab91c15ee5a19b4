#!/bin/bash
# Round 3: flash64 (D = 64 v1-structure kernel with pre-scaled Q, -m through the MFMA, max-free fast path).
# Attention GPU tests first, then the whole suite, the attention lab, the SD2.1 bench with flash64 on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or attn" --timeout 120 \
  --timeout-method thread > gpurun_out/r3a_pytest_attn.log 2>&1 || { tail -30 gpurun_out/r3a_pytest_attn.log; exit 1; }
tail -1 gpurun_out/r3a_pytest_attn.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3a_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3a_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3a_pytest_gpu.log
timeout -k 10 300 ./tools/gemm_lab/bin/attn_lab > gpurun_out/r3a_attn_lab.log 2>&1 || { tail -20 gpurun_out/r3a_attn_lab.log; exit 1; }
grep -v stamps gpurun_out/r3a_attn_lab.log
timeout -k 10 500 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3a_bench_sd21.log 2>&1 || exit $?
echo "== sd21 flash64"; tail -1 gpurun_out/r3a_bench_sd21.log | cut -c1-300
SHAI_FLASH64=0 timeout -k 10 500 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3a_bench_sd21_off.log 2>&1 || exit $?
echo "== sd21 flash64 off"; tail -1 gpurun_out/r3a_bench_sd21_off.log | cut -c1-300
