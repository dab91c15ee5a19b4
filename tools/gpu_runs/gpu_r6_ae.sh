#!/bin/bash
# Round 6: merged FF down + proj_out on the unfolded (batch-1) path too -- tests, tune, SD2.1 b1 p50 merged vs not.
# tune the new keys, then SD2.1 b32 merged vs not (SHAI_MERGE_PROJ_OUT), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sd_gpu.py tests/test_norm_handoff_gpu.py tests/test_step_batching_gpu.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/r6ae_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6ae_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6ae_tests.log | head; exit $rc; }
cp config/gemm_tuning_mi355x.json gpurun_out/tune_r6ae.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6ae.json
SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6ae.json timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --latency-runs 2 \
  > gpurun_out/r6ae_tune.log 2>&1 || { tail -5 gpurun_out/r6ae_tune.log; exit 1; }
for rep in 1 2; do
  for arm in 1 0; do
    SHAI_MERGE_PROJ_OUT=$arm timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --latency-runs 5 > gpurun_out/r6ae_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6ae_sd_$arm$rep.log; exit 1; }
    echo "merge=$arm rep $rep: $(grep '^{' gpurun_out/r6ae_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
