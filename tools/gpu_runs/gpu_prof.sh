#!/bin/bash
# rocprofv3 kernel trace of one bench step (after warm-up); markdown summary -> gpurun_out/prof_<workload>.md
# usage: bash tools/gpu_runs/gpu_prof.sh <sd21|mistral|flux|mllama> [extra bench.py args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WL=${1:-sd21}
shift || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$WL -o run --output-format csv -- \
  python3 bench.py --workload $WL --steps 1 --warmup 1 --latency-runs 0 "$@" > gpurun_out/prof_$WL.log 2>&1
rc=$?
tail -3 gpurun_out/prof_$WL.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_$WL -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$(dirname $f)" 40 "$WL" > gpurun_out/prof_$WL.md
find gpurun_out/prof_$WL -name '*kernel_trace.csv' -delete
head -30 gpurun_out/prof_$WL.md
