#!/bin/bash
# Round 6: halo-tiled GroupNorm conv routing at SD2.1 batch 1 (SHAI_HALO_CONV 0 / 1 / 2; measured slower at b32),
# b1 p50 alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in 1 2 0; do
    SHAI_HALO_CONV=$arm timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --latency-runs 7 > gpurun_out/r6ah_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6ah_sd_$arm$rep.log; exit 1; }
    echo "halo=$arm rep $rep: $(grep '^{' gpurun_out/r6ah_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
