#!/bin/bash
# Round-3 closing evidence on one MI355X: GPU suite, smoke(), the driver's default SD2.1 bench line (20 / 5 as the
# driver runs it), the other workloads' lines (Mistral, Flux, ViT, mllama, SD2.1 768^2), then a kernel profile of
# one SD2.1 batch.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3z_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3z_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3z_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3z_smoke.log 2>&1 || { tail -20 gpurun_out/r3z_smoke.log; exit 1; }
tail -1 gpurun_out/r3z_smoke.log | cut -c1-300
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3z_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r3z_bench_sd21.log
for wl in mistral flux vit mllama t5; do
  timeout -k 10 500 python -u bench.py --workload $wl > gpurun_out/r3z_bench_$wl.log 2>&1 || exit $?
  echo "== $wl"; tail -1 gpurun_out/r3z_bench_$wl.log
done
timeout -k 10 500 python -u bench.py --height 768 --width 768 --batch 16 --steps 3 --warmup 1 \
  > gpurun_out/r3z_bench_sd21_768.log 2>&1 || exit $?
echo "== sd21 768"; tail -1 gpurun_out/r3z_bench_sd21_768.log
bash tools/rocprof.sh r3z_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 > /dev/null || exit 1
head -30 gpurun_out/rocprof_r3z_sd21.md
