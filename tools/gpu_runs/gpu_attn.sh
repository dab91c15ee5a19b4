# flash-attention A/B: numerics tests, then the attention microbench with the 32- and 64-query-per-wave forms
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "flash or attn" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1 || { tail -30 gpurun_out/pytest_attn.log; exit 1; }
tail -2 gpurun_out/pytest_attn.log
SHAI_ATTN_QB=1 timeout -k 10 300 python -u tools/bench_kernels.py --only attn > gpurun_out/kb_attn_qb1.log 2>&1 && grep attn gpurun_out/kb_attn_qb1.log
SHAI_ATTN_QB=2 timeout -k 10 300 python -u tools/bench_kernels.py --only attn > gpurun_out/kb_attn_qb2.log 2>&1 && grep attn gpurun_out/kb_attn_qb2.log
