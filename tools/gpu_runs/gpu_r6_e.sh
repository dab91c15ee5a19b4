#!/bin/bash
# Round 6 evidence on the current tree: the SD2.1 batch-32 bench line, then rocprofv3 kernel traces of one SD2.1
# batch-32 step (50 UNet steps + text encoder + VAE) and of the Mistral-7B b64 decode bench, summarised on the box
# with tools/prof_db.py (warm tuning cache: the shipped config/gemm_tuning_mi355x.json, autotune off in the trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6e_bench.log 2>&1 || { tail -20 gpurun_out/r6e_bench.log; exit 1; }
grep '^{' gpurun_out/r6e_bench.log | tail -1 | cut -c1-300
prof() {  # name, title, bench args...
  local name=$1 title=$2; shift 2
  SHAI_GEMM_AUTOTUNE=0 timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r6e_$name -o run -- python3 -u bench.py "$@" \
    > gpurun_out/r6e_$name.log 2>&1 || { tail -20 gpurun_out/r6e_$name.log; return 1; }
  grep '^{' gpurun_out/r6e_$name.log | tail -1 | cut -c1-300
  python3 tools/prof_db.py $(find gpurun_out/r6e_$name -name "*results.db" | head -1) --top 40 --title "$title" \
    > gpurun_out/r6e_$name.md && rm -rf gpurun_out/r6e_$name
  head -12 gpurun_out/r6e_$name.md
}
prof sd21 "SD2.1 512^2 batch 32, one bench step (round 6 final tree)" --steps 1 --warmup 1 --latency-runs 0 || exit 1
prof mistral "Mistral-7B b64 decode, one bench step (round 6 final tree)" --workload mistral --steps 1 --warmup 1 || exit 1
