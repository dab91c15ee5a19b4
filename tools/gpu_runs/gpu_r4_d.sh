#!/bin/bash
# Round 4: SD2.1 b32 kernel profile on the round-4 tree, and an end-to-end A/B of the register-staged flash64
# (SHAI_FLASH64_DMA=0) against the LDS-DMA one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/rocprof.sh r4d_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 || exit $?
timeout -k 10 400 python -u bench.py --gpus 1 --steps 4 --warmup 1 --latency-runs 0 > gpurun_out/r4d_bench_dma.log 2>&1 || exit $?
echo "dma: $(tail -1 gpurun_out/r4d_bench_dma.log | cut -c1-200)"
SHAI_FLASH64_DMA=0 timeout -k 10 400 python -u bench.py --gpus 1 --steps 4 --warmup 1 --latency-runs 0 > gpurun_out/r4d_bench_nodma.log 2>&1 || exit $?
echo "reg: $(tail -1 gpurun_out/r4d_bench_nodma.log | cut -c1-200)"
