#!/bin/bash
# Round-3 closing kernel profiles of ViT-b16 batch 32 and Mistral-7B b64 decode on the final tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/rocprof.sh r3_vit -- bench.py --workload vit --steps 20 --warmup 2 --latency-runs 0 > /dev/null || exit 1
head -32 gpurun_out/rocprof_r3_vit.md
bash tools/rocprof.sh r3_mistral -- bench.py --workload mistral --steps 1 --warmup 1 > /dev/null || exit 1
head -32 gpurun_out/rocprof_r3_mistral.md
