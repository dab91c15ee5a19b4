#!/bin/bash
# Round 5: re-race the SD2.1 batch-32 shapes after the round-5 kernel changes, then A/B the bench on the old / new cache
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_runs/gpu_retune_subset.sh 'any(s in key for s in ("262144", ":65536,", ":16384,", "|64,"))' \
  "--workload sd21 --steps 1 --warmup 1 --latency-runs 0" || exit 1
cp gpurun_out/tune_subset.json gpurun_out/r5u_tune.json
for f in config/gemm_tuning_mi355x.json gpurun_out/r5u_tune.json config/gemm_tuning_mi355x.json gpurun_out/r5u_tune.json; do
  SHAI_GEMM_TUNE_FILE=$f SHAI_GEMM_AUTOTUNE=0 timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 --latency-runs 0 \
    > gpurun_out/r5u_bench.log 2>&1 || { tail -20 gpurun_out/r5u_bench.log; exit 1; }
  echo "$f: $(tail -1 gpurun_out/r5u_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
