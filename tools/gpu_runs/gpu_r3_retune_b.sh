#!/bin/bash
# Round 3 retune, part B: start from part A's cache (config/gemm_tuning_r3a.json: SD2.1 shapes re-measured) and
# re-add the Flux / mllama / ViT / Mistral shapes part A dropped.  Result: gpurun_out/tune_b.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=gpurun_out/tune_b.json
cp config/gemm_tuning_r3a.json $OUT
export SHAI_GEMM_TUNE_FILE=$OUT SHAI_GEMM_TUNE_SAVE=$OUT
i=0
for args in "--workload flux --steps 1 --warmup 1 --latency-runs 1" "--workload mllama --steps 1 --warmup 1 --latency-runs 1" \
            "--workload vit --steps 1 --warmup 1" "--workload mistral --steps 1 --warmup 1 --batch 64" \
            "--workload mistral --steps 1 --warmup 1 --batch 32"; do
  i=$((i + 1))
  timeout -k 10 600 python -u bench.py $args > gpurun_out/retune_b_$i.log 2>&1
  rc=$?
  echo "[$i] rc=$rc $(tail -1 gpurun_out/retune_b_$i.log | cut -c1-200)"
  [ $rc -eq 0 ] || exit $rc
done
python3 -c "import json,collections;e=json.load(open('$OUT'));print(len(e),'entries',dict(collections.Counter(x.rsplit('=',1)[1].split(',')[0] for x in e)))"
