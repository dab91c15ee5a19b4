#!/bin/bash
# skinny2 with coalesced split-K slabs and the 6-stage ring: numerics, per-shape sweep (v1 vs v2 variants vs
# the cold-cache tuner's pick), Mistral b64 decode re-tuned cold with the choices saved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gpu.py -m gpu -x -q -k "skinny2" --timeout 120 --timeout-method thread \
  > gpurun_out/r3_s2b_tests.log 2>&1 || { tail -40 gpurun_out/r3_s2b_tests.log; exit 1; }
tail -1 gpurun_out/r3_s2b_tests.log
SHAI_DECODE_M=1,64 SHAI_NUM_CFGS=0 timeout -k 10 400 python -u tools/bench_kernels.py --only decode > gpurun_out/r3_s2b_decode.log 2>&1 || { tail -20 gpurun_out/r3_s2b_decode.log; exit 1; }
grep decode_gemm gpurun_out/r3_s2b_decode.log
SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_cold2.json timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_s2b_mistral.log 2>&1 || { tail -20 gpurun_out/r3_s2b_mistral.log; exit 1; }
echo "== mistral"; tail -1 gpurun_out/r3_s2b_mistral.log | cut -c1-300
