#!/bin/bash
# flash2 d64 with pre-scaled Q / max-folded accumulators: attention numerics, TF/s table, ViT profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or attn" --timeout 120 --timeout-method thread \
  > gpurun_out/r3_attn_tests.log 2>&1 || { tail -40 gpurun_out/r3_attn_tests.log; exit 1; }
tail -1 gpurun_out/r3_attn_tests.log
timeout -k 10 300 python -u tools/bench_kernels.py --only attn > gpurun_out/r3_attn_bench.log 2>&1 || { tail -20 gpurun_out/r3_attn_bench.log; exit 1; }
grep "op=attn" gpurun_out/r3_attn_bench.log
bash tools/rocprof.sh vit_b32 -- bench.py --workload vit --steps 5 --warmup 2 || exit $?
