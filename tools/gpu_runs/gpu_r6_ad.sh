#!/bin/bash
# Round 6: Transformer2D input GroupNorm folded into proj_in per image (weight slices on the v4 kernel) -- tests, tune,
# then SD2.1 b32 folded vs not (SHAI_GN_FOLD_PROJ_IN), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_sd_gpu.py tests/test_norm_handoff_gpu.py -q -x \
  -k "slices or sd or handoff or unet or conv2d" --timeout 300 --timeout-method thread > gpurun_out/r6ad_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6ad_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6ad_tests.log | head; exit $rc; }
cp config/gemm_tuning_mi355x.json gpurun_out/tune_r6ad.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6ad.json
SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6ad.json timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --latency-runs 2 \
  > gpurun_out/r6ad_tune.log 2>&1 || { tail -5 gpurun_out/r6ad_tune.log; exit 1; }
for rep in 1 2; do
  for arm in 1 0; do
    SHAI_GN_FOLD_PROJ_IN=$arm timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 --latency-runs 3 > gpurun_out/r6ad_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6ad_sd_$arm$rep.log; exit 1; }
    echo "fold=$arm rep $rep: $(grep '^{' gpurun_out/r6ad_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
