#!/bin/bash
# Round 4, second GPU call: the tests touched this round, the GPU suite, smoke, SD2.1 bench lines (labs: gpu_r4_a.sh)
# decode tests touched this round (staged fused reduce, default two-shot routing, partials placeholder,
# 64k / 128k decode attention), then the whole GPU suite, smoke, a short SD2.1 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py tests/test_skinny_gpu.py tests/test_kernels_gpu.py -k "p2p or tp2 or skinny or qkv or d512 or long_context or decode" -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/r4a_pytest_p2p.log 2>&1 || { tail -40 gpurun_out/r4a_pytest_p2p.log; exit 1; }
tail -3 gpurun_out/r4a_pytest_p2p.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4a_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4a_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4a_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.log 2>&1 || { tail -20 gpurun_out/r4a_smoke.log; exit 1; }
tail -1 gpurun_out/r4a_smoke.log | cut -c1-300
timeout -k 10 400 python -u bench.py --gpus 1 --steps 8 --warmup 2 > gpurun_out/r4a_bench_sd21.log 2>&1 || exit $?
tail -1 gpurun_out/r4a_bench_sd21.log | cut -c1-400
# A/B: GroupNorm finalize fused into the stats launch (ticket) at batch 1 latency
SHAI_GN_FUSED_FINALIZE=1 timeout -k 10 400 python -u bench.py --gpus 1 --steps 1 --warmup 1 --latency-runs 5 > gpurun_out/r4a_bench_gnfused.log 2>&1 || exit $?
echo "gn fused finalize: $(tail -1 gpurun_out/r4a_bench_gnfused.log | grep -o '"p50_latency_ms_bs1": [0-9.]*')"
