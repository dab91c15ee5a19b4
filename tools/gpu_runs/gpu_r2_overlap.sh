#!/bin/bash
# Row-parallel compute / communication overlap on two ranks sharing one GPU (P2P all-reduce, HIP graph).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_p2p_gpu.py -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/r2o_tests.log 2>&1 || { tail -40 gpurun_out/r2o_tests.log; exit 1; }
tail -1 gpurun_out/r2o_tests.log
