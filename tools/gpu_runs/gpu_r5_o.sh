#!/bin/bash
# Round 5: retire hipBLASLt -- drop the 48 library entries of the tuning cache and re-race those shapes on the
# hand-written kernels (library path off by default now) through every workload that produces them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_runs/gpu_retune_subset.sh 'cfg == 2000' \
  "--workload flux --height 512 --width 512 --steps 1 --warmup 1 --inference-steps 2 --latency-runs 0" \
  "--workload flux --height 1024 --width 1024 --steps 1 --warmup 1 --inference-steps 2 --latency-runs 0" \
  "--workload mllama --steps 1 --warmup 1" \
  "--workload vit --steps 2 --warmup 1" \
  "--workload t5 --steps 1 --warmup 1" \
  "--workload mistral --steps 1 --warmup 1 --gen-len 8" \
  "--workload sd21 --steps 1 --warmup 1 --latency-runs 1" || exit 1
cp gpurun_out/tune_subset.json gpurun_out/r5o_tune.json
