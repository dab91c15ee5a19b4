#!/bin/bash
# Round 6: phase conv with split-K (the fold maps GEMM rows to output pixels) -- forced-config tests, then SD2.1
# with the phase conv on every eligible upsample conv (SHAI_UP2_MIN_TILES=0: batch-1 shapes too, split-K) vs the
# 256-tile threshold, alternating; b1 p50 is the number to watch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm3_gpu.py tests/test_kernels_gpu.py -q -x -k "up2 or upsample" \
  --timeout 300 --timeout-method thread > gpurun_out/r6z_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6z_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6z_tests.log | head; exit $rc; }
cp config/gemm_tuning_mi355x.json gpurun_out/tune_r6z.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6z.json SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6z.json
for rep in 1 2; do
  for mt in 0 256; do
    SHAI_UP2_MIN_TILES=$mt timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --latency-runs 5 > gpurun_out/r6z_sd_$mt$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6z_sd_$mt$rep.log; exit 1; }
    echo "min_tiles=$mt rep $rep: $(grep '^{' gpurun_out/r6z_sd_$mt$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
