#!/bin/bash
# Round 6: Mistral-7B b64, o_proj / down as the in-launch split-K fixup (tools/gpu_runs/tune_fixup_ab.json) vs the
# shipped cache (skinny + fold launch), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for arm in shipped fixup; do
    f=config/gemm_tuning_mi355x.json; [ $arm = fixup ] && f=tools/gpu_runs/tune_fixup_ab.json
    SHAI_GEMM_TUNE_FILE=$f timeout -k 10 600 python -u bench.py --workload mistral --steps 3 > gpurun_out/r6q_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6q_$arm$rep.log; exit 1; }
    echo "$arm $rep: $(grep '^{' gpurun_out/r6q_$arm$rep.log | tail -1 | grep -o '"value": [0-9.]*')"
  done
done
