#!/bin/bash
# Round 5: decode baseline -- per-shape decode GEMM race (M = 64), Mistral-7B b64 bench line, kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_DECODE_M=64 timeout -k 10 300 python -u tools/bench_kernels.py --only decode > gpurun_out/r5j_decode.log 2>&1 || { tail -20 gpurun_out/r5j_decode.log; exit 1; }
grep -v Warning gpurun_out/r5j_decode.log | tail -8 | cut -c1-400
timeout -k 10 300 python -u bench.py --workload mistral --steps 2 --warmup 1 > gpurun_out/r5j_mistral.log 2>&1 || { tail -20 gpurun_out/r5j_mistral.log; exit 1; }
tail -1 gpurun_out/r5j_mistral.log | cut -c1-600
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5j_prof -o r5j -- python3 -u bench.py --workload mistral --steps 1 --warmup 1 > gpurun_out/r5j_prof.log 2>&1 || { tail -20 gpurun_out/r5j_prof.log; exit 1; }
find gpurun_out/r5j_prof -name "*kernel_stats.csv" | head -3
