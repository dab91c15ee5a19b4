#!/bin/bash
# Round 6: the v2 kernel's in-launch split-K fixup (SHAI_G2_FIXUP=1, round 4: slower) re-measured at SD2.1 batch 1
# against the fold launch, alternating (b1 p50 is the number; b32 rides along).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in 1 0; do
    SHAI_G2_FIXUP=$arm timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --latency-runs 7 > gpurun_out/r6af_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6af_sd_$arm$rep.log; exit 1; }
    echo "g2fixup=$arm rep $rep: $(grep '^{' gpurun_out/r6af_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
