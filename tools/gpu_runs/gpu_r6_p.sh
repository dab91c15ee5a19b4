#!/bin/bash
# Round 6: SD2.1 batch-1 latency (50 steps) A/B of the GroupNorm statistics routes: producer hand-off partials
# (col_partials fallback + gn_from_partials, default) vs standalone stats with the finalize fused into the stats
# launch (SHAI_NORM_HANDOFF=0 SHAI_GN_FUSED_FINALIZE=1), alternating, 4 timed generates each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --batch 1 --steps 4 --warmup 1 --latency-runs 0 > gpurun_out/r6p_$name.log 2>&1 \
    || { tail -5 gpurun_out/r6p_$name.log; return 1; }
  echo "$name: $(grep '^{' gpurun_out/r6p_$name.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
}
for rep in 1 2; do
  run A_default_$rep SHAI_X=0 || exit 1
  run B_nohandoff_fused_$rep SHAI_NORM_HANDOFF=0 SHAI_GN_FUSED_FINALIZE=1 || exit 1
  run C_handoff_fused_$rep SHAI_GN_FUSED_FINALIZE=1 || exit 1
  run D_nohandoff_$rep SHAI_NORM_HANDOFF=0 || exit 1
done
