#!/bin/bash
# Round 4: in-launch split-K fixup for the v2 tile GEMM (cfg 2-4): forced-split tests, the GEMM / conv / SD suites,
# SD2.1 b32 + bs1 latency with the fixup on vs off (SHAI_G2_FIXUP=0), and a batch-1 profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "splitk or fixup" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r4h_pytest_fixup.log 2>&1 || { tail -30 gpurun_out/r4h_pytest_fixup.log; exit 1; }
tail -1 gpurun_out/r4h_pytest_fixup.log
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm3_gpu.py tests/test_sd_gpu.py tests/test_skinny_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r4h_pytest_rel.log 2>&1 || { tail -30 gpurun_out/r4h_pytest_rel.log; exit 1; }
tail -1 gpurun_out/r4h_pytest_rel.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 3 --warmup 1 --latency-runs 5 > gpurun_out/r4h_bench_on.log 2>&1 || exit $?
echo "fixup on:  $(tail -1 gpurun_out/r4h_bench_on.log | cut -c1-160) $(tail -1 gpurun_out/r4h_bench_on.log | grep -o '"p50_latency_ms_bs1": [0-9.]*')"
SHAI_G2_FIXUP=0 timeout -k 10 400 python -u bench.py --gpus 1 --steps 3 --warmup 1 --latency-runs 5 > gpurun_out/r4h_bench_off.log 2>&1 || exit $?
echo "fixup off: $(tail -1 gpurun_out/r4h_bench_off.log | cut -c1-160) $(tail -1 gpurun_out/r4h_bench_off.log | grep -o '"p50_latency_ms_bs1": [0-9.]*')"
bash tools/rocprof.sh r4h_sd21_bs1 -- bench.py --batch 1 --steps 3 --warmup 1 --latency-runs 0 || exit $?
