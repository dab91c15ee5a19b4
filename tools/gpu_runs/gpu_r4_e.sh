#!/bin/bash
# Round 4: norm hand-offs (GroupNorm partials / LayerNorm moments from the GEMM epilogue, LayerNorm folded into
# the consuming projection): new GPU tests, the GEMM / conv / SD suites they touch, then SD2.1 b32 with the
# hand-offs on vs off (SHAI_NORM_HANDOFF=0) and a kernel profile of the hand-off build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_norm_handoff_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4e_pytest_handoff.log 2>&1 || { tail -40 gpurun_out/r4e_pytest_handoff.log; exit 1; }
tail -2 gpurun_out/r4e_pytest_handoff.log
timeout -k 10 600 python -u -m pytest tests/test_gemm3_gpu.py tests/test_kernels_gpu.py tests/test_sd_gpu.py tests/test_models_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r4e_pytest_rel.log 2>&1 || { tail -30 gpurun_out/r4e_pytest_rel.log; exit 1; }
tail -1 gpurun_out/r4e_pytest_rel.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 4 --warmup 1 --latency-runs 3 > gpurun_out/r4e_bench_on.log 2>&1 || exit $?
echo "handoff on:  $(tail -1 gpurun_out/r4e_bench_on.log | cut -c1-200) $(tail -1 gpurun_out/r4e_bench_on.log | grep -o '"p50_latency_ms_bs1": [0-9.]*')"
SHAI_NORM_HANDOFF=0 timeout -k 10 400 python -u bench.py --gpus 1 --steps 4 --warmup 1 --latency-runs 3 > gpurun_out/r4e_bench_off.log 2>&1 || exit $?
echo "handoff off: $(tail -1 gpurun_out/r4e_bench_off.log | cut -c1-200) $(tail -1 gpurun_out/r4e_bench_off.log | grep -o '"p50_latency_ms_bs1": [0-9.]*')"
bash tools/rocprof.sh r4e_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 || exit $?
