#!/bin/bash
# Re-measure the tuning-cache entries selected by a Python predicate over (key, cfg, splits), then run
# the given bench workloads so those shapes are raced again against every config (including ones added
# since they were measured).  Result: gpurun_out/tune_subset.json (full cache) -> review, then merge.
#   bash tools/gpu_runs/gpu_retune_subset.sh '<predicate>' "<bench args>" ["<bench args>" ...]
# e.g. bash tools/gpu_runs/gpu_retune_subset.sh 'cfg in (9, 10)' "--workload sd21 --steps 1 --warmup 1 --latency-runs 0"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/tune_subset.json
PRED=$1; shift
python3 - "$OUT" "$PRED" <<'PY'
import json, sys
e = json.load(open("config/gemm_tuning_mi355x.json"))
keep = []
for x in e:
    key, v = x.rsplit("=", 1)
    cfg, splits = (int(t) for t in v.split(","))
    if not eval(sys.argv[2], {}, {"key": key, "cfg": cfg, "splits": splits}):
        keep.append(x)
json.dump(keep, open(sys.argv[1], "w"), indent=0)
print(f"kept {len(keep)} of {len(e)} entries; {len(e) - len(keep)} to re-measure")
PY
export SHAI_GEMM_TUNE_FILE=$OUT SHAI_GEMM_TUNE_SAVE=$OUT
i=0
for args in "$@"; do
  i=$((i + 1))
  timeout -k 10 900 python -u bench.py $args > gpurun_out/retune_subset_$i.log 2>&1
  rc=$?
  echo "[$i] rc=$rc $(tail -1 gpurun_out/retune_subset_$i.log | cut -c1-220)"
  [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" <<'PY'
import json, sys, collections
e = json.load(open(sys.argv[1]))
print(len(e), "entries;", dict(collections.Counter(x.rsplit("=", 1)[1].split(",")[0] for x in e)))
PY
