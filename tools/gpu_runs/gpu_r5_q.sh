#!/bin/bash
# Round 5: A/B of the hipBLASLt retirement -- each workload on the round-4 cache with the library path on vs the
# re-raced cache with it off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in "--workload flux --height 1024 --width 1024 --steps 1 --warmup 1 --inference-steps 4 --latency-runs 0" \
          "--workload flux --height 512 --width 512 --steps 2 --warmup 1 --inference-steps 4 --latency-runs 0" \
          "--workload mllama --steps 2 --warmup 1" "--workload vit --steps 5 --warmup 2" "--workload t5 --steps 5 --warmup 2" \
          "--workload mistral --steps 1 --warmup 1 --gen-len 16"; do
  a=$(SHAI_GEMM_LIB=1 SHAI_GEMM_TUNE_FILE=config/ab_old_tune.json SHAI_GEMM_AUTOTUNE=0 timeout -k 10 600 python -u bench.py $wl 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('p50_ttft_ms',''))") || exit 1
  b=$(SHAI_GEMM_AUTOTUNE=0 timeout -k 10 600 python -u bench.py $wl 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('p50_ttft_ms',''))") || exit 1
  echo "$wl | lib(r4 cache): $a | hand-written(r5 cache): $b" | tee -a gpurun_out/r5q_ab.log
done
