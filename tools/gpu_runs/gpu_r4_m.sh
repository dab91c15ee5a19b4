#!/bin/bash
# Round 4: re-race the SD2.1 GEMM / conv shapes now that the four-wave kernel (cfg 13) exists and the v4 epilogue
# carries the norm hand-offs, then A/B the SD2.1 b32 line with the shipped cache vs the re-tuned one (same box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 60; do echo "running $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/gpu_runs/gpu_retune_subset.sh 'cfg in (9, 10, 11, 12, 13)' \
  "--steps 1 --warmup 1 --latency-runs 0" || exit $?
for c in shipped tuned shipped tuned; do
  if [ $c = shipped ]; then F=config/gemm_tuning_mi355x.json; else F=gpurun_out/tune_subset.json; fi
  SHAI_GEMM_TUNE_FILE=$F SHAI_GEMM_AUTOTUNE=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --latency-runs 0 \
    > gpurun_out/r4m_sd_$c.log 2>&1 || exit $?
  echo "$c: $(tail -1 gpurun_out/r4m_sd_$c.log | cut -c1-130)"
done
