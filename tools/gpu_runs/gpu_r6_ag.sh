#!/bin/bash
# Round 6: ResNet shortcut conv forked onto a side stream at small batch (graph branches replay concurrently,
# tools/probes/graph_branches.py) -- SD GPU tests, then SD2.1 b1 p50 forked vs not (SHAI_SD_FORK), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sd_gpu.py tests/test_step_batching_gpu.py tests/test_norm_handoff_gpu.py tests/test_models_gpu.py -q -x \
  --timeout 300 --timeout-method thread > gpurun_out/r6ag_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6ag_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6ag_tests.log | head; exit $rc; }
for rep in 1 2; do
  for arm in 1 0; do
    SHAI_SD_FORK=$arm timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --latency-runs 7 > gpurun_out/r6ag_sd_$arm$rep.log 2>&1 \
      || { tail -5 gpurun_out/r6ag_sd_$arm$rep.log; exit 1; }
    echo "fork=$arm rep $rep: $(grep '^{' gpurun_out/r6ag_sd_$arm$rep.log | tail -1 | grep -o "\"value\": [0-9.]*\|\"p50_latency_ms_bs1\": [0-9.]*" | tr "\n" " ")"
  done
done
