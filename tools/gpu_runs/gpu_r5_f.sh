#!/bin/bash
# Round 5: W-stationary kernel (GLU: interleaved epilogue; plain / residual: per-tile epilogue) -- lab, forced tests,
# re-race of the cached K = 320 plain GEMM shapes with cfg 15 as a candidate, SD2.1 bench line on the re-raced cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab --ws > gpurun_out/r5f_lab.log 2>&1 || { cat gpurun_out/r5f_lab.log; exit 1; }
grep -E "==|v4_320w |ws_" gpurun_out/r5f_lab.log | grep -v "OK$"
grep -c MISMATCH gpurun_out/r5f_lab.log || true
timeout -k 10 300 python -u -m pytest tests/test_gemm_ws_gpu.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/r5f_pytest.log 2>&1 || { tail -30 gpurun_out/r5f_pytest.log; exit 1; }
tail -1 gpurun_out/r5f_pytest.log
bash tools/gpu_runs/gpu_retune_subset.sh '",320,b1" in key and key.startswith("0:")' \
  "--workload sd21 --steps 1 --warmup 1 --latency-runs 0" || exit 1
cp gpurun_out/tune_subset.json gpurun_out/r5f_tune.json
SHAI_GEMM_TUNE_FILE=gpurun_out/r5f_tune.json timeout -k 10 600 python -u bench.py --steps 8 --warmup 2 \
  > gpurun_out/r5f_bench.log 2>&1 || { tail -20 gpurun_out/r5f_bench.log; exit 1; }
tail -1 gpurun_out/r5f_bench.log | cut -c1-400
python3 - <<'PY'
import json
e = json.load(open("gpurun_out/r5f_tune.json"))
for x in e:
    if ",320,b1" in x and x.startswith("0:"):
        print(x)
PY
