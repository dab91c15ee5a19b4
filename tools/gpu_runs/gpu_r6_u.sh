#!/bin/bash
# Round 6: phase-decomposed upsample conv (v4 CONV 3) -- conv numerics tests, tune its new GEMM keys into a copy of
# the shipped cache through the SD2.1 bench, then SD2.1 b32 with the phase conv on / off (alternating), and a
# kernel-stats profile of the phase-conv arm.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_conv_halo_gpu.py tests/test_norm_handoff_gpu.py \
  -q -x -k "conv or handoff or unet" --timeout 120 --timeout-method thread > gpurun_out/r6u_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6u_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6u_tests.log | head; exit $rc; }
cp config/gemm_tuning_mi355x.json gpurun_out/tune_r6u.json
SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6u.json SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6u.json \
  timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/r6u_tune.log 2>&1 || { tail -5 gpurun_out/r6u_tune.log; exit 1; }
echo "tune: $(grep '^{' gpurun_out/r6u_tune.log | tail -1 | cut -c1-200)"
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6u.json
for rep in 1 2; do
  for arm in 1 0; do
    SHAI_UP2_PHASES=$arm timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 > gpurun_out/r6u_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6u_sd_$arm$rep.log; exit 1; }
    echo "phases=$arm rep $rep: $(grep '^{' gpurun_out/r6u_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r6u_prof -o r6u -- python3 -u bench.py --steps 2 --warmup 1 \
  > gpurun_out/r6u_prof.log 2>&1 || { tail -5 gpurun_out/r6u_prof.log; exit 1; }
echo prof ok
