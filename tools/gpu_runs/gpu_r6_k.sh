#!/bin/bash
# Round 6: forced v2 tile-config tests; Mistral-7B b64 decode bench with the wave-per-block decode attention on / off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm3_gpu.py -q -x -k "every_tile_config" --timeout 120 \
  --timeout-method thread > gpurun_out/r6k_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6k_tests.log; [ $rc -eq 0 ] || exit $rc
for wb in 1 0; do
  SHAI_DECODE_WB=$wb timeout -k 10 600 python -u bench.py --workload mistral > gpurun_out/r6k_mistral_wb$wb.log 2>&1 \
    || { tail -5 gpurun_out/r6k_mistral_wb$wb.log; exit 1; }
  echo "wb=$wb $(grep '^{' gpurun_out/r6k_mistral_wb$wb.log | tail -1 | cut -c1-260)"
done
