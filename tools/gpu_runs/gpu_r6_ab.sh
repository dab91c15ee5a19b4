#!/bin/bash
# Round 6: few-output-channel conv kernel (conv_smalln.hip: UNet / VAE conv_out) -- conv tests, then SD2.1 b32 with
# it on / off (SHAI_CONV_SMALLN), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_sd_gpu.py -q -x -k "conv or vae or sd or unet" \
  --timeout 300 --timeout-method thread > gpurun_out/r6ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6ab_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6ab_tests.log | head; exit $rc; }
for rep in 1 2; do
  for arm in 1 0; do
    SHAI_CONV_SMALLN=$arm timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 --latency-runs 3 > gpurun_out/r6ab_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6ab_sd_$arm$rep.log; exit 1; }
    echo "smalln=$arm rep $rep: $(grep '^{' gpurun_out/r6ab_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
