#!/bin/bash
# Round 6: halo-tiled GroupNorm-fused conv -- numerics vs fp32, kernel A/B at the SD2.1 shapes, the SD model tests,
# and the bench line with the fused path on.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_halo_gpu.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/r6b_halo_tests.log 2>&1 || { tail -40 gpurun_out/r6b_halo_tests.log; exit 1; }
tail -2 gpurun_out/r6b_halo_tests.log
timeout -k 10 400 python -u tools/bench_halo.py --out gpurun_out/r6b_halo_bench.json > gpurun_out/r6b_halo_bench.log 2>&1 \
  || { tail -20 gpurun_out/r6b_halo_bench.log; exit 1; }
cat gpurun_out/r6b_halo_bench.log | cut -c1-400
timeout -k 10 600 python -u -m pytest tests/test_sd_gpu.py tests/test_norm_handoff_gpu.py tests/test_models_gpu.py -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/r6b_pytest.log 2>&1 || { tail -40 gpurun_out/r6b_pytest.log; exit 1; }
tail -2 gpurun_out/r6b_pytest.log
timeout -k 10 600 python -u bench.py --steps 6 --warmup 2 > gpurun_out/r6b_bench.log 2>&1 || { tail -20 gpurun_out/r6b_bench.log; exit 1; }
grep '^{' gpurun_out/r6b_bench.log | tail -1 | cut -c1-300
