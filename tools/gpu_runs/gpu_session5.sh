set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for b in 16 32; do
  timeout -k 10 600 python -u bench.py --batch $b --steps 2 --warmup 1 --latency-runs 0 > gpurun_out/bench_b$b.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_b$b.log | cut -c1-200
done
timeout -k 10 300 python -u tools/bench_kernels.py --only attn,norm,sdgemm > gpurun_out/kbench.log 2>&1 || exit $?
cat gpurun_out/kbench.log
