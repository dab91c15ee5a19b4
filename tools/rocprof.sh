#!/bin/bash
# Kernel-level profile of any python entry point:
#   bash tools/rocprof.sh <name> [--pmc "COUNTERS"] -- <python args...>
# e.g.
#   bash tools/rocprof.sh sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0
#   bash tools/rocprof.sh gemm_pmc --pmc "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CU_CYCLES" -- tools/bench_kernels.py --only gemm
# Pass 1 (always): --kernel-trace --stats -> gpurun_out/rocprof_<name>/ + markdown summary
#   gpurun_out/rocprof_<name>.md (hand-written shai:: kernels appear by name).
# Pass 2 (optional, its own run -- never combined with other trace domains): --pmc counters, hard-killed
#   after 120 s (a counter set the hardware cannot collect hangs rocprofv3).
# Copy the summaries worth keeping into profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NAME=$1; shift
PMC=""
if [ "$1" = "--pmc" ]; then PMC=$2; shift 2; fi
[ "$1" = "--" ] && shift
OUT=gpurun_out/rocprof_$NAME
mkdir -p "$OUT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- python3 "$@" \
  > "$OUT.log" 2>&1
rc=$?
tail -3 "$OUT.log"
[ $rc -eq 0 ] || exit $rc
f=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$(dirname "$f")" 40 "$NAME" > "$OUT.md"
find "$OUT" -name '*kernel_trace.csv' -delete
head -25 "$OUT.md"
if [ -n "$PMC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $PMC -d "${OUT}_pmc" -o run --output-format csv -- python3 "$@" \
    > "${OUT}_pmc.log" 2>&1 || exit $?
  find "${OUT}_pmc" -name '*counter_collection.csv' | head -1
fi
