#!/bin/bash
# Decode GEMM choice with the read-flush cold tuner (median of 5 cold launches): per-shape table, Mistral b64
# bench re-tuned with the choices saved, then a kernel-trace profile of the bench on the saved choices.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_DECODE_M=1,64 SHAI_NUM_CFGS=0 timeout -k 10 400 python -u tools/bench_kernels.py --only decode > gpurun_out/r3_dp_decode.log 2>&1 || { tail -20 gpurun_out/r3_dp_decode.log; exit 1; }
grep decode_gemm gpurun_out/r3_dp_decode.log
SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_cold3.json timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_dp_mistral.log 2>&1 || { tail -20 gpurun_out/r3_dp_mistral.log; exit 1; }
echo "== mistral (tuned cold)"; tail -1 gpurun_out/r3_dp_mistral.log | cut -c1-400
SHAI_GEMM_TUNE_FILE=gpurun_out/tune_cold3.json timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_dp_mistral2.log 2>&1 || { tail -20 gpurun_out/r3_dp_mistral2.log; exit 1; }
echo "== mistral (saved choices)"; tail -1 gpurun_out/r3_dp_mistral2.log | cut -c1-400
SHAI_GEMM_TUNE_FILE=gpurun_out/tune_cold3.json bash tools/rocprof.sh mistral_b64_r3 -- bench.py --workload mistral --steps 2 --warmup 1 || exit $?
