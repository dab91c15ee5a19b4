#!/bin/bash
# Kernel-level session: fp8 GEMM (all three tiles), decode-attention microbench, decode gate_up PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_runs/gpu_r3_f8.sh || exit $?
timeout -k 10 300 python -u tools/bench_kernels.py --only dattn > gpurun_out/r3_dattn.log 2>&1 || { tail -20 gpurun_out/r3_dattn.log; exit 1; }
grep "op=" gpurun_out/r3_dattn.log
bash tools/gpu_runs/gpu_r3_pmc.sh || exit $?
