#!/bin/bash
# GPU check after the mllama + GroupNorm-grid changes: targeted tests, SD2.1 profile, mllama bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mllama_gpu.py tests/test_kernels_gpu.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/pytest_s2.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_s2.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_runs/gpu_prof.sh sd21 || exit $?
timeout -k 10 600 python -u bench.py --workload mllama --steps 1 --warmup 1 --latency-runs 2 --batch 8 \
  > gpurun_out/bench_mllama.log 2>&1
rc=$?
tail -2 gpurun_out/bench_mllama.log
exit $rc
