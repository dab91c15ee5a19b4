#!/bin/bash
# Round-2 closing evidence on one MI355X: full GPU test suite, smoke(), the driver's default SD2.1 bench line,
# Mistral / Flux / ViT bench lines.  Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r2f_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r2f_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r2f_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2f_smoke.log 2>&1 || { tail -20 gpurun_out/r2f_smoke.log; exit 1; }
tail -1 gpurun_out/r2f_smoke.log | cut -c1-300
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2f_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r2f_bench_sd21.log | cut -c1-400
for wl in mistral flux vit; do
  timeout -k 10 500 python -u bench.py --workload $wl > gpurun_out/r2f_bench_$wl.log 2>&1 || exit $?
  echo "== $wl"; tail -1 gpurun_out/r2f_bench_$wl.log | cut -c1-400
done
