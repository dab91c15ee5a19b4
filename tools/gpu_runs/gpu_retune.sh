# Autotune the bench workloads' shapes missing from config/gemm_tuning_mi355x.json;
# result gpurun_out/gemm_tuning_mi355x.json (merge over config/ afterwards with tools/merge_tuning.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
# NOTE: gpurun_out/ is not shipped to the box: start from the committed config instead
cp config/gemm_tuning_mi355x.json gpurun_out/gemm_tuning_mi355x.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/gemm_tuning_mi355x.json SHAI_GEMM_TUNE_SAVE=gpurun_out/gemm_tuning_mi355x.json
for spec in "sd21:--workload sd21 --batch 16 --steps 1 --warmup 1 --latency-runs 1" \
            "flux:--workload flux --steps 1 --warmup 1 --latency-runs 1" \
            "mllama:--workload mllama --steps 1 --warmup 1 --latency-runs 1" \
            "mistral64:--workload mistral --steps 1 --warmup 1 --batch 64" \
            "mistral32:--workload mistral --steps 1 --warmup 1 --batch 32"; do
  wl=${spec%%:*}; args=${spec#*:}
  timeout -k 10 900 python -u bench.py $args > gpurun_out/retune_$wl.log 2>&1
  rc=$?
  echo "$wl rc=$rc"; tail -1 gpurun_out/retune_$wl.log | cut -c1-220
  [ $rc -eq 0 ] || exit $rc
done
