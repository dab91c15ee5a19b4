#!/bin/bash
# GroupNorm apply with one channel vector per thread: GN / UNet tests, kernel timing, SD2.1 bench line + profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_sd_gpu.py tests/test_models_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3n_pytest.log 2>&1 || { tail -30 gpurun_out/r3n_pytest.log; exit 1; }
tail -1 gpurun_out/r3n_pytest.log
timeout -k 10 300 python -u tools/bench_kernels.py --only norm > gpurun_out/r3n_norm.log 2>&1 || { tail -20 gpurun_out/r3n_norm.log; exit 1; }
grep -i "group" gpurun_out/r3n_norm.log | head -12
timeout -k 10 500 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3n_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r3n_bench_sd21.log | cut -c1-250
bash tools/rocprof.sh r3n_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 > /dev/null || exit 1
grep -E "gn_|Total" gpurun_out/rocprof_r3n_sd21.md
