#!/bin/bash
# Mistral-7B b64 decode evidence: engine / skinny / sampler GPU tests (also with the X-in-registers skinny
# variant), bench lines (async decode, sync decode, XR skinny), a kernel-trace profile of the bench and the
# decode-GEMM bandwidth table for both skinny variants.  Each GPU step has its own time limit; stop at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="--timeout 120 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_skinny_gpu.py -x -q $T -k "engine or skinny or sampler" \
  > gpurun_out/llm_gpu_tests.log 2>&1 || { tail -30 gpurun_out/llm_gpu_tests.log; exit 1; }
tail -1 gpurun_out/llm_gpu_tests.log
SHAI_SKINNY_XR=1 timeout -k 10 400 python -u -m pytest tests/test_skinny_gpu.py -x -q $T -k "skinny" \
  > gpurun_out/skinny_xr_tests.log 2>&1 || { tail -30 gpurun_out/skinny_xr_tests.log; exit 1; }
echo "== XR tests"; tail -1 gpurun_out/skinny_xr_tests.log
SHAI_DECODE_M=64 SHAI_NUM_CFGS=0 timeout -k 10 300 python -u tools/bench_kernels.py --only decode > gpurun_out/kbench_decode64.log 2>&1 || exit $?
grep decode_gemm gpurun_out/kbench_decode64.log | cut -c1-200
SHAI_SKINNY_XR=1 SHAI_DECODE_M=64 SHAI_NUM_CFGS=0 timeout -k 10 300 python -u tools/bench_kernels.py --only decode > gpurun_out/kbench_decode64_xr.log 2>&1 || exit $?
echo "== XR"; grep decode_gemm gpurun_out/kbench_decode64_xr.log | cut -c1-200
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/bench_mistral_async.log 2>&1 || exit $?
echo "== mistral async"; tail -1 gpurun_out/bench_mistral_async.log | cut -c1-700
SHAI_SKINNY_XR=1 timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/bench_mistral_xr.log 2>&1 || exit $?
echo "== mistral async XR"; tail -1 gpurun_out/bench_mistral_xr.log | cut -c1-700
SHAI_ASYNC_DECODE=0 timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/bench_mistral_sync.log 2>&1 || exit $?
echo "== mistral sync"; tail -1 gpurun_out/bench_mistral_sync.log | cut -c1-700
bash tools/rocprof.sh mistral_b64 -- bench.py --workload mistral --steps 2 --warmup 1 || exit $?
