#!/bin/bash
# Wide skinny decode GEMM (gemv2.hip): numerics tests, per-shape bandwidth vs the first skinny kernel,
# Mistral b64 decode with and without it in the tuner.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gpu.py -m gpu -x -q -k "skinny2" --timeout 120 --timeout-method thread \
  > gpurun_out/r3_s2_tests.log 2>&1 || { tail -40 gpurun_out/r3_s2_tests.log; exit 1; }
tail -1 gpurun_out/r3_s2_tests.log
SHAI_DECODE_M=1,64 SHAI_NUM_CFGS=0 timeout -k 10 300 python -u tools/bench_kernels.py --only decode > gpurun_out/r3_s2_decode.log 2>&1 || { tail -20 gpurun_out/r3_s2_decode.log; exit 1; }
grep decode_gemm gpurun_out/r3_s2_decode.log
for s2 in 1 0; do
  SHAI_SKINNY2=$s2 timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_mistral_s2_$s2.log 2>&1 || { tail -20 gpurun_out/r3_mistral_s2_$s2.log; exit 1; }
  echo "== mistral skinny2=$s2"; tail -1 gpurun_out/r3_mistral_s2_$s2.log | cut -c1-330
done
