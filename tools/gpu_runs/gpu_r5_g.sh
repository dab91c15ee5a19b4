#!/bin/bash
# Round 5: producer-side LayerNorm (ws LNO epilogue) -- tests, re-race of the K = 320 shapes, SD2.1 bench line,
# per-op breakdown of one UNet step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_ws_gpu.py tests/test_norm_handoff_gpu.py tests/test_gemm3_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r5g_pytest.log 2>&1 || { tail -30 gpurun_out/r5g_pytest.log; exit 1; }
tail -1 gpurun_out/r5g_pytest.log
bash tools/gpu_runs/gpu_retune_subset.sh '",320,b1" in key and key.startswith("0:")' \
  "--workload sd21 --steps 1 --warmup 1 --latency-runs 0" || exit 1
cp gpurun_out/tune_subset.json gpurun_out/r5g_tune.json
SHAI_GEMM_TUNE_FILE=gpurun_out/r5g_tune.json timeout -k 10 600 python -u bench.py --steps 8 --warmup 2 \
  > gpurun_out/r5g_bench.log 2>&1 || { tail -20 gpurun_out/r5g_bench.log; exit 1; }
tail -1 gpurun_out/r5g_bench.log | cut -c1-300
python3 - <<'PY'
import json
for x in json.load(open("gpurun_out/r5g_tune.json")):
    if ",320,b1" in x and x.startswith("0:"):
        print(x)
PY
SHAI_GEMM_TUNE_FILE=gpurun_out/r5g_tune.json timeout -k 10 300 python -u tools/op_breakdown.py --batch 32 --top 40 \
  > gpurun_out/r5g_opbreak.log 2>&1 || { tail -20 gpurun_out/r5g_opbreak.log; exit 1; }
grep -v Warning gpurun_out/r5g_opbreak.log | head -30 | cut -c1-150
