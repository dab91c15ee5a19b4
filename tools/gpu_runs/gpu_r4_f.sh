#!/bin/bash
# Round 4: hand-off fixes (one wave per (image, group) GroupNorm finalize, folding only when the consumer GEMMs fill
# the chip): hand-off tests, SD2.1 b32 + bs1 latency, ViT-b16 b32 with the hand-offs on vs off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_norm_handoff_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1 || { tail -30 gpurun_out/r4f_pytest.log; exit 1; }
tail -1 gpurun_out/r4f_pytest.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 4 --warmup 1 --latency-runs 5 > gpurun_out/r4f_bench_sd.log 2>&1 || exit $?
echo "sd: $(tail -1 gpurun_out/r4f_bench_sd.log | cut -c1-200) $(tail -1 gpurun_out/r4f_bench_sd.log | grep -o '"p50_latency_ms_bs1": [0-9.]*')"
timeout -k 10 300 python -u bench.py --workload vit --steps 20 --warmup 3 > gpurun_out/r4f_vit_on.log 2>&1 || exit $?
echo "vit handoff on:  $(tail -1 gpurun_out/r4f_vit_on.log | cut -c1-160)"
SHAI_NORM_HANDOFF=0 timeout -k 10 300 python -u bench.py --workload vit --steps 20 --warmup 3 > gpurun_out/r4f_vit_off.log 2>&1 || exit $?
echo "vit handoff off: $(tail -1 gpurun_out/r4f_vit_off.log | cut -c1-160)"
