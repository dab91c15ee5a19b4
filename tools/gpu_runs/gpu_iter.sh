# quick GPU iteration: kernel tests, norm/attention microbench, SD bench (each step time-limited)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_sd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1 || { tail -30 gpurun_out/pytest_k.log; exit 1; }
tail -2 gpurun_out/pytest_k.log
timeout -k 10 600 python -u tools/bench_kernels.py --only ${KB:-attn,norm} > gpurun_out/kb.log 2>&1 && grep -E "attn|groupnorm|gemm|conv" gpurun_out/kb.log
for b in ${BATCHES:-16}; do
timeout -k 10 600 python -u bench.py --batch $b > gpurun_out/bench_sd_b$b.log 2>&1 && tail -1 gpurun_out/bench_sd_b$b.log | cut -c1-250 || exit 1
done
