#!/bin/bash
# Round 6: Flux.1-dev 1024^2 with the phase-decomposed VAE upsample convs on / off (alternating, shipped cache).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in 1 0; do
    SHAI_UP2_PHASES=$arm timeout -k 10 600 python -u bench.py --workload flux --height 1024 --width 1024 --steps 3 --warmup 1 \
      > gpurun_out/r6w_$arm$rep.log 2>&1 || { tail -5 gpurun_out/r6w_$arm$rep.log; exit 1; }
    echo "phases=$arm rep $rep: $(grep '^{' gpurun_out/r6w_$arm$rep.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  done
done
