#!/bin/bash
# Round 6: the LayerNorm-fold threshold (SHAI_FOLD_MIN_TILES, 192) now that the folded Transformer2D path also
# merges FF-down into proj_out and folds the GroupNorm into proj_in: 64 (the 8x8 mid block folded too) vs 192, b32.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp config/gemm_tuning_mi355x.json gpurun_out/tune_r6aj.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6aj.json
SHAI_FOLD_MIN_TILES=64 SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6aj.json timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --latency-runs 1 \
  > gpurun_out/r6aj_tune.log 2>&1 || { tail -5 gpurun_out/r6aj_tune.log; exit 1; }
for rep in 1 2; do
  for mt in 64 192; do
    SHAI_FOLD_MIN_TILES=$mt timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 --latency-runs 1 > gpurun_out/r6aj_sd_$mt$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6aj_sd_$mt$rep.log; exit 1; }
    echo "fold_min=$mt rep $rep: $(grep '^{' gpurun_out/r6aj_sd_$mt$rep.log | tail -1 | grep -o "\"value\": [0-9.]*")"
  done
done
