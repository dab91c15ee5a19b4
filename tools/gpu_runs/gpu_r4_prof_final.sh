#!/bin/bash
# Round 4: SD2.1 b32 kernel profile of the closing tree (hand-offs, retuned cache).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/rocprof.sh r4z_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 > /dev/null || exit 1
head -40 gpurun_out/rocprof_r4z_sd21.md
