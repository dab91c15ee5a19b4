#!/bin/bash
# Paged decode attention split-K A/B on the Mistral-7B b64 bench (SHAI_DECODE_WG = target workgroups).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for wg in 512 1024 2048; do
  SHAI_DECODE_WG=$wg timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r2d_bench_$wg.log 2>&1 || exit $?
  echo "== WG $wg"; tail -1 gpurun_out/r2d_bench_$wg.log | cut -c1-80; tail -1 gpurun_out/r2d_bench_$wg.log | grep -o '"p50_tpot_ms.*'
done
SHAI_DECODE_WG=1024 bash tools/rocprof.sh r2d_mistral_1024 -- bench.py --workload mistral --steps 2 --warmup 1 > /dev/null || exit $?
grep -n "decode_attn\|decode_combine" gpurun_out/rocprof_r2d_mistral_1024.md
