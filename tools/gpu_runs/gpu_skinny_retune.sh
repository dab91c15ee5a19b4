#!/bin/bash
# Re-measure every skinny-eligible (M <= 64) GEMM of the decode workloads with both split-K forms (separate
# fold / in-kernel fixup) racing; result gpurun_out/tune_skinny.json -> merge over config/gemm_tuning_mi355x.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/tune_skinny.json
python3 - "$OUT" <<'PY'
import json, sys
e = json.load(open("config/gemm_tuning_mi355x.json"))
keep = [x for x in e if int(x.split(":", 1)[1].split(",", 1)[0]) > 64]
json.dump(keep, open(sys.argv[1], "w"), indent=0)
print(f"kept {len(keep)} of {len(e)} entries (dropped M <= 64)")
PY
export SHAI_GEMM_TUNE_FILE=$OUT SHAI_GEMM_TUNE_SAVE=$OUT
for spec in "mistral64:--workload mistral --steps 3 --warmup 1 --batch 64" \
            "mistral32:--workload mistral --steps 1 --warmup 1 --batch 32" \
            "mllama:--workload mllama --steps 1 --warmup 1 --latency-runs 1" \
            "flux:--workload flux --steps 1 --warmup 1 --latency-runs 0"; do
  wl=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 python -u bench.py $args > gpurun_out/skt_$wl.log 2>&1
  rc=$?
  echo "$wl rc=$rc $(tail -1 gpurun_out/skt_$wl.log | cut -c1-170)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --workload mistral --steps 3 --warmup 1 --batch 64 > gpurun_out/skt_final64.log 2>&1 || exit $?
tail -1 gpurun_out/skt_final64.log | cut -c1-200
python3 -c "
import json; e=json.load(open('$OUT')); print(sum('=1100,' in x for x in e), 'fixup picks;', sum('=1000,' in x for x in e), 'fold picks')"
