#!/bin/bash
# Round 4: re-race the tuned GEMM shapes whose cached choice is a v4 tile config or hipBLASLt against every config
# (now including the four-wave 256 x 256 kernel, cfg 13) on the LLM / Flux / ViT / mllama / T5 workloads.
# Output: gpurun_out/tune_subset.json (kept entries + re-measured ones); merged over the shipped cache afterwards
# with tools/merge_tuning.py (entries of shapes not re-run keep their old choice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 60; do echo "retune running $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
bash tools/gpu_runs/gpu_retune_subset.sh 'cfg in (9, 10, 11, 12, 2000)' \
  "--workload flux --steps 1 --warmup 1" \
  "--workload mistral --steps 1 --warmup 1" \
  "--workload vit --steps 2 --warmup 1" \
  "--workload t5 --steps 2 --warmup 1" \
  "--workload mllama --steps 1 --warmup 1" || exit $?
python3 - <<'PY'
import json, collections
e = json.load(open("gpurun_out/tune_subset.json"))
w4 = [x for x in e if x.rsplit("=", 1)[1].split(",")[0] == "13"]
print(len(w4), "shapes now on the four-wave kernel:")
for x in w4: print("  ", x)
PY
