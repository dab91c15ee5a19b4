#!/bin/bash
# Re-measure the whole GEMM tuning cache from scratch (every shape of the bench workloads races every tile
# config, including ones added since the committed cache was measured); result
# gpurun_out/gemm_tuning_fresh.json -> copy over config/gemm_tuning_mi355x.json after review.
# Then one SD2.1 bench on the fresh cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/gemm_tuning_fresh.json
echo "[]" > $OUT
export SHAI_GEMM_TUNE_FILE=$OUT SHAI_GEMM_TUNE_SAVE=$OUT
for spec in "sd21:--workload sd21 --steps 1 --warmup 1 --latency-runs 1" \
            "sd21b16:--workload sd21 --batch 16 --steps 1 --warmup 1 --latency-runs 0" \
            "flux:--workload flux --steps 1 --warmup 1 --latency-runs 1" \
            "mllama:--workload mllama --steps 1 --warmup 1 --latency-runs 1" \
            "mistral64:--workload mistral --steps 1 --warmup 1 --batch 64" \
            "mistral32:--workload mistral --steps 1 --warmup 1 --batch 32"; do
  wl=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 python -u bench.py $args > gpurun_out/retune_$wl.log 2>&1
  rc=$?
  echo "$wl rc=$rc entries=$(python3 -c "import json;print(len(json.load(open('$OUT'))))")"
  tail -1 gpurun_out/retune_$wl.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/retune_sd21_bench.log 2>&1 || exit $?
tail -1 gpurun_out/retune_sd21_bench.log | cut -c1-300
