#!/bin/bash
# Round 5: batch-1 GroupNorm chain fusions (statistics + apply in one launch for few images; split-K folds write the
# GroupNorm partials) -- norm / kernel tests, batch-1 A/B (split-K fold GroupNorm partials off / on), SD2.1 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_norm_handoff_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r5s_pytest.log 2>&1 || { tail -30 gpurun_out/r5s_pytest.log; exit 1; }
tail -1 gpurun_out/r5s_pytest.log
for v in 0 1; do
  SHAI_FOLD_GN=$v timeout -k 10 300 python -u bench.py --batch 1 --steps 3 --warmup 1 --latency-runs 3 > gpurun_out/r5s_b1_$v.log 2>&1 || { tail -20 gpurun_out/r5s_b1_$v.log; exit 1; }
  echo "fold_gn=$v: $(tail -1 gpurun_out/r5s_b1_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('p50_latency_ms_bs1'))")"
done
timeout -k 10 600 python -u bench.py --steps 8 --warmup 2 > gpurun_out/r5s_bench.log 2>&1 || { tail -20 gpurun_out/r5s_bench.log; exit 1; }
tail -1 gpurun_out/r5s_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('p50_latency_ms_bs1'))"
