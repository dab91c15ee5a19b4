#!/bin/bash
# Round 4: split-K fixup v2 (batched slab loads, 256x128 / 128x64 tiles only): tests, SD2.1 bs1 latency on vs off,
# then a kernel profile of the long-context scenario (32k prompt beside 16 decoders) to locate the long TPOT.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "splitk or fixup" -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r4i_pytest_fixup.log 2>&1 || { tail -30 gpurun_out/r4i_pytest_fixup.log; exit 1; }
tail -1 gpurun_out/r4i_pytest_fixup.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 1 --warmup 1 --latency-runs 7 > gpurun_out/r4i_bench_on.log 2>&1 || exit $?
echo "fixup on:  $(tail -1 gpurun_out/r4i_bench_on.log | grep -o '"p50_latency_ms_bs1": [0-9.]*') $(tail -1 gpurun_out/r4i_bench_on.log | cut -c1-120)"
SHAI_G2_FIXUP=0 timeout -k 10 400 python -u bench.py --gpus 1 --steps 1 --warmup 1 --latency-runs 7 > gpurun_out/r4i_bench_off.log 2>&1 || exit $?
echo "fixup off: $(tail -1 gpurun_out/r4i_bench_off.log | grep -o '"p50_latency_ms_bs1": [0-9.]*') $(tail -1 gpurun_out/r4i_bench_off.log | cut -c1-120)"
bash tools/rocprof.sh r4i_long -- -m shai_amd.bench.long_context --model llama31_8b --prompt-len 32768 --chunk 8192 \
  --background 16 --gen 64 || exit $?
