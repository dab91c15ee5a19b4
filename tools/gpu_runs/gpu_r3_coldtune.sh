#!/bin/bash
# Decode GEMM autotune with cold (Infinity-Cache-flushed) timings: Mistral b64 decode re-tuned from the
# shipped cache (M<=64 entries absent), with the tuner's new choices saved; vs the round-2 warm-tuned cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_cold.json timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_cold_a.log 2>&1 || { tail -20 gpurun_out/r3_cold_a.log; exit 1; }
echo "== cold-tuned"; tail -1 gpurun_out/r3_cold_a.log | cut -c1-300
SHAI_GEMM_TUNE_FILE=gpurun_out/tune_cold.json timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_cold_b.log 2>&1 || { tail -20 gpurun_out/r3_cold_b.log; exit 1; }
echo "== cold-tuned cache reload"; tail -1 gpurun_out/r3_cold_b.log | cut -c1-300
SHAI_GEMM_TUNE_FILE=config/ab/old_tune.json timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_cold_c.log 2>&1 || { tail -20 gpurun_out/r3_cold_c.log; exit 1; }
echo "== round-2 cache"; tail -1 gpurun_out/r3_cold_c.log | cut -c1-300
SHAI_DECODE_M=1,64 SHAI_NUM_CFGS=0 timeout -k 10 300 python -u tools/bench_kernels.py --only decode > gpurun_out/r3_cold_dec.log 2>&1 || { tail -20 gpurun_out/r3_cold_dec.log; exit 1; }
grep decode_gemm gpurun_out/r3_cold_dec.log
