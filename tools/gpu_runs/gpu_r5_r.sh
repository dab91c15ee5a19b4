#!/bin/bash
# Round 5 evidence: rocprofv3 kernel traces of Flux 512^2 / 1024^2, SD2.1 batch 1 and ViT b32 on a warm tuning
# cache (a tune pass of each workload first, saved to gpurun_out/r5r_tune.json; the profiled pass runs with
# SHAI_GEMM_AUTOTUNE=0 so no autotune sweep lands in the trace), summarised with tools/prof_db.py on the box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp config/gemm_tuning_mi355x.json gpurun_out/r5r_tune.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/r5r_tune.json SHAI_GEMM_TUNE_SAVE=gpurun_out/r5r_tune.json
prof() {  # name, title, bench args...
  local name=$1 title=$2; shift 2
  timeout -k 10 400 python3 -u bench.py "$@" > gpurun_out/r5r_${name}_tune.log 2>&1 || { tail -20 gpurun_out/r5r_${name}_tune.log; return 1; }
  SHAI_GEMM_AUTOTUNE=0 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r5r_$name -o run -- python3 -u bench.py "$@" \
    > gpurun_out/r5r_$name.log 2>&1 || { tail -20 gpurun_out/r5r_$name.log; return 1; }
  grep '^{' gpurun_out/r5r_$name.log | tail -1 | cut -c1-240
  python3 tools/prof_db.py $(find gpurun_out/r5r_$name -name "*results.db" | head -1) --top 30 --title "$title" \
    > gpurun_out/r5r_$name.md && rm -rf gpurun_out/r5r_$name
}
prof flux512 "Flux.1-dev 512^2, 28 steps (round 5)" --workload flux --height 512 --width 512 --steps 1 --warmup 1 \
  --inference-steps 28 --latency-runs 0 || exit 1
prof flux1024 "Flux.1-dev 1024^2, 28 steps (round 5)" --workload flux --height 1024 --width 1024 --steps 1 --warmup 1 \
  --inference-steps 28 --latency-runs 0 || exit 1
prof sdb1 "SD2.1 batch 1, 50 steps (round 5)" --batch 1 --steps 2 --warmup 1 --latency-runs 0 || exit 1
prof vit "ViT-base/16 batch 32 (round 5)" --workload vit --steps 20 --warmup 3 || exit 1
