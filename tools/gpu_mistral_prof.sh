#!/bin/bash
# Mistral-7B b64 decode evidence: kernel-trace profile of the bench and decode-GEMM bandwidth table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/rocprof.sh mistral_b64 -- bench.py --workload mistral --steps 2 --warmup 1 || exit $?
SHAI_DECODE_M=64 SHAI_NUM_CFGS=0 timeout -k 10 300 python -u tools/bench_kernels.py --only decode > gpurun_out/kbench_decode64.log 2>&1 || exit $?
cat gpurun_out/kbench_decode64.log | grep decode_gemm
