#!/bin/bash
# Round 6: tune the phase-decomposed upsample conv's GEMM keys of the Flux VAE (512^2 / 1024^2) into a copy of the
# shipped cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp config/gemm_tuning_mi355x.json gpurun_out/tune_r6v.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6v.json SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6v.json
for spec in "flux512:--workload flux --steps 1 --warmup 1" "flux1024:--workload flux --height 1024 --width 1024 --steps 1 --warmup 1"; do
  wl=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 python -u bench.py $args > gpurun_out/r6v_$wl.log 2>&1 || { tail -5 gpurun_out/r6v_$wl.log; exit 1; }
  echo "$wl: $(grep '^{' gpurun_out/r6v_$wl.log | tail -1 | cut -c1-260)"
done
