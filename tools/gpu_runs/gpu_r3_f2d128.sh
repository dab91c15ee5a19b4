#!/bin/bash
# flash2 D = 128 with the immediate-offset reads, pre-scaled Q and the -m MFMA: attention tests, attention lab
# (f2-prev = the previous D = 128 M segment), Flux 512^2 / 1024^2 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_varlen_gpu.py tests/test_flux_gpu.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/r3d_pytest.log 2>&1 || { tail -30 gpurun_out/r3d_pytest.log; exit 1; }
tail -1 gpurun_out/r3d_pytest.log
timeout -k 10 300 ./tools/gemm_lab/bin/attn_lab > gpurun_out/r3d_attn_lab.log 2>&1 || { tail -20 gpurun_out/r3d_attn_lab.log; exit 1; }
grep -v stamps gpurun_out/r3d_attn_lab.log
timeout -k 10 500 python -u bench.py --workload flux > gpurun_out/r3d_flux.log 2>&1 || exit $?
echo "== flux 512"; tail -1 gpurun_out/r3d_flux.log | cut -c1-250
timeout -k 10 600 python -u bench.py --workload flux --height 1024 --width 1024 --steps 2 --warmup 1 --latency-runs 1 \
  > gpurun_out/r3d_flux1024.log 2>&1 || exit $?
echo "== flux 1024"; tail -1 gpurun_out/r3d_flux1024.log | cut -c1-250
