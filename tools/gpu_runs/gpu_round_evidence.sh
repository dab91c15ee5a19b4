#!/bin/bash
# Round-end evidence on one MI355X: kernel-vs-library microbenchmarks, the Flux / mllama / fp8 benches and a
# rocprofv3 kernel-trace of the Mistral decode bench.  Every GPU step has its own time limit; the script stops
# at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_kernels.py > gpurun_out/kbench_all.log 2>&1 || exit $?
echo "== kbench ok"
for wl in flux mllama; do
  timeout -k 10 600 python -u bench.py --workload $wl > gpurun_out/bench_$wl.log 2>&1 || exit $?
  echo "== $wl"; tail -1 gpurun_out/bench_$wl.log | cut -c1-400
done
timeout -k 10 600 python -u bench.py --workload mistral --quantization fp8 > gpurun_out/bench_mistral_fp8.log 2>&1 || exit $?
echo "== mistral fp8"; tail -1 gpurun_out/bench_mistral_fp8.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mistral -o run -- python3 bench.py --workload mistral --steps 2 --warmup 1 > gpurun_out/prof_mistral.log 2>&1 || exit $?
echo "== prof ok"
