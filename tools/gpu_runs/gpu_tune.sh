#!/bin/bash
# Accumulate the GEMM autotuner cache over every bench workload (each run loads the file, autotunes the
# shapes it has not seen, saves the union) -> gpurun_out/gemm_tuning_mi355x.json; copy to config/ after.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=gpurun_out/gemm_tuning_mi355x.json
[ -f "$T" ] || cp config/gemm_tuning_mi355x.json "$T" 2>/dev/null || true
export SHAI_GEMM_TUNE_FILE=$T SHAI_GEMM_TUNE_SAVE=$T
for wl in "$@"; do
  case $wl in
    sd21)    args="--workload sd21 --steps 1 --warmup 1 --latency-runs 1" ;;
    mistral) args="--workload mistral --steps 1 --warmup 1 --batch 32" ;;
    mistral64) args="--workload mistral --steps 1 --warmup 1 --batch 64" ;;
    flux)    args="--workload flux --steps 1 --warmup 1 --latency-runs 1 --batch 1" ;;
    mllama)  args="--workload mllama --steps 1 --warmup 1 --latency-runs 1 --batch 8" ;;
  esac
  timeout -k 10 900 python -u bench.py $args > gpurun_out/tune_$wl.log 2>&1
  rc=$?
  echo "$wl rc=$rc"; tail -1 gpurun_out/tune_$wl.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
