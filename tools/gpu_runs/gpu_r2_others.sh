#!/bin/bash
# Round-2 measurement of the non-headline workloads + a Flux kernel profile.  Each GPU step has its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in flux mistral mllama; do
  timeout -k 10 400 python -u bench.py --workload $wl > gpurun_out/r2_bench_$wl.log 2>&1 || exit $?
  echo "== $wl"; tail -1 gpurun_out/r2_bench_$wl.log | cut -c1-330
done
bash tools/rocprof.sh r2_flux -- bench.py --workload flux --steps 1 --warmup 1 --latency-runs 0 || exit $?
