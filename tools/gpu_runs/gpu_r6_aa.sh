#!/bin/bash
# Round 6: phase conv over image groups (H W < 256, e.g. the UNet's 8 -> 16 upsample conv) -- phase-conv tests
# (forced configs, split-K, grouped shapes), tune the new key, then SD2.1 b32 with the 8 -> 16 conv phased
# (SHAI_UP2_MIN_TILES=256, shipped) vs not (400), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm3_gpu.py tests/test_kernels_gpu.py -q -x -k "up2 or upsample" \
  --timeout 300 --timeout-method thread > gpurun_out/r6aa_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6aa_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6aa_tests.log | head; exit $rc; }
cp config/gemm_tuning_mi355x.json gpurun_out/tune_r6aa.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6aa.json
SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6aa.json timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --latency-runs 1 \
  > gpurun_out/r6aa_tune.log 2>&1 || { tail -5 gpurun_out/r6aa_tune.log; exit 1; }
for rep in 1 2; do
  for mt in 256 400; do
    SHAI_UP2_MIN_TILES=$mt timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 --latency-runs 1 > gpurun_out/r6aa_sd_$mt$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6aa_sd_$mt$rep.log; exit 1; }
    echo "min_tiles=$mt rep $rep: $(grep '^{' gpurun_out/r6aa_sd_$mt$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
