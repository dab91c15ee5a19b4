#!/bin/bash
# Round 5: Mistral b64 decode A/B of the fusion toggles (qkv fold inside attention, fused RoPE/KV-write decode)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for env in "SHAI_QKV_FOLD_IN_ATTN=1" "SHAI_QKV_FOLD_IN_ATTN=0" "SHAI_QKV_FOLD_MAX_SPLITS=0" "SHAI_QKV_FOLD_IN_ATTN=1"; do
  env $env timeout -k 10 400 python -u bench.py --workload mistral --steps 2 --warmup 1 > gpurun_out/r5v.log 2>&1 || { tail -20 gpurun_out/r5v.log; exit 1; }
  echo "$env: $(tail -1 gpurun_out/r5v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_tpot_ms'])")"
done
