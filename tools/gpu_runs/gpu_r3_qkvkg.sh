#!/bin/bash
# K-group count of the QKV partials folded inside decode attention: tuned (fold) value vs 2 / 4 / 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for kg in 0 2 4 8 0 2 4 8; do
  SHAI_QKV_PART_KG=$kg timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/qk_$kg.log 2>&1 || exit $?
  echo "kg=$kg $(tail -1 gpurun_out/qk_$kg.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_tpot_ms"])')"
done
