#!/bin/bash
# Round 6: Mistral-7B b64 decode kernel trace on the current tree with the shipped tuning cache (compare with
# profiles/mistral7b_b64_kernels_round6.md, taken before the skinny kernel's 16-B reduction / epilogue).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_GEMM_AUTOTUNE=0 timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r6o_m -o run -- python3 -u bench.py \
  --workload mistral --steps 1 --warmup 1 > gpurun_out/r6o_m.log 2>&1 || { tail -20 gpurun_out/r6o_m.log; exit 1; }
grep '^{' gpurun_out/r6o_m.log | tail -1 | cut -c1-200
python3 tools/prof_db.py $(find gpurun_out/r6o_m -name "*results.db" | head -1) --top 12 \
  --title "Mistral-7B b64 decode, skinny 16-B epilogue (round 6)" > gpurun_out/r6o_m.md && rm -rf gpurun_out/r6o_m
head -18 gpurun_out/r6o_m.md
