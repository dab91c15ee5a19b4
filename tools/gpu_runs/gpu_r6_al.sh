#!/bin/bash
# Round 6: re-race every SD2.1 GEMM / conv key from scratch on the closing kernels (an empty cache through the b32
# bench and its batch-1 latency runs), then SD2.1 b32 on the fresh SD keys (merged over the shipped cache) vs the
# shipped cache, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "[]" > gpurun_out/tune_r6al_sd.json
SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6al_sd.json SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6al_sd.json \
  timeout -k 10 900 python -u bench.py --steps 1 --warmup 1 --latency-runs 1 > gpurun_out/r6al_tune.log 2>&1 \
  || { tail -5 gpurun_out/r6al_tune.log; exit 1; }
python3 - <<'PY'
import json
old = json.load(open("config/gemm_tuning_mi355x.json"))
new = json.load(open("gpurun_out/tune_r6al_sd.json"))
key = lambda e: e.rsplit("=", 1)[0]
fresh = {key(e): e for e in new}
merged = [fresh.pop(key(e), e) for e in old] + list(fresh.values())
json.dump(merged, open("gpurun_out/tune_r6al_merged.json", "w"), indent=0)
changed = sum(1 for e in old if key(e) in {key(x) for x in new} and e not in set(new))
print(f"fresh SD keys {len(new)}, changed choices {changed}, merged {len(merged)}")
PY
for rep in 1 2; do
  for arm in fresh shipped; do
    f=config/gemm_tuning_mi355x.json; [ $arm = fresh ] && f=gpurun_out/tune_r6al_merged.json
    SHAI_GEMM_TUNE_FILE=$f timeout -k 10 600 python -u bench.py --steps 4 --warmup 1 --latency-runs 3 > gpurun_out/r6al_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6al_sd_$arm$rep.log; exit 1; }
    echo "$arm rep $rep: $(grep '^{' gpurun_out/r6al_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
