#!/bin/bash
# Round 6: ViT classification with the last layer's query side for the CLS token only -- encoder GPU tests, the
# graph-replayed A/B against the full encoder (tools/probes/vit_cls_ab.py), then the ViT b32 bench line twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py -q -x -k "encoder or vit" --timeout 300 --timeout-method thread \
  > gpurun_out/r6ai_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6ai_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r6ai_tests.log | head; exit $rc; }
timeout -k 10 300 python -u tools/probes/vit_cls_ab.py 2>&1 | grep -v amdgpu.ids
for rep in 1 2; do
  timeout -k 10 600 python -u bench.py --workload vit > gpurun_out/r6ai_vit$rep.log 2>&1 || { tail -5 gpurun_out/r6ai_vit$rep.log; exit 1; }
  echo "vit rep $rep: $(grep '^{' gpurun_out/r6ai_vit$rep.log | tail -1 | grep -o '"value": [0-9.]*')"
done
