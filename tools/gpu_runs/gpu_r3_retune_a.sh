#!/bin/bash
# Round 3 retune, part A: drop every cached tile-GEMM / conv choice with M >= 2048 (the wide-epilogue v4 kernel
# changed the race), re-measure them through the SD2.1 b32 and b16 benches.  Result: gpurun_out/tune_subset.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/gpu_runs/gpu_retune_subset.sh '(cfg < 1000 or cfg == 2000) and int(key.split(":")[1].split(",")[0]) >= 2048' \
  "--workload sd21 --steps 1 --warmup 1 --latency-runs 0" \
  "--workload sd21 --batch 16 --steps 1 --warmup 1 --latency-runs 0"
rc=$?; [ $rc -eq 0 ] || exit $rc
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_subset.json
timeout -k 10 500 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3t_bench_sd21.log 2>&1 || exit $?
echo "== sd21 retuned"; tail -1 gpurun_out/r3t_bench_sd21.log | cut -c1-300
bash tools/rocprof.sh r3t_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 > /dev/null || exit 1
head -36 gpurun_out/rocprof_r3t_sd21.md
