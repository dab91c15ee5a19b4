#!/bin/bash
# Round-4 closing evidence (2/2): the other workloads' lines (Mistral, Flux, ViT, mllama, T5, SD2.1 768^2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in mistral flux vit mllama t5; do
  timeout -k 10 400 python -u bench.py --workload $wl > gpurun_out/r4z_bench_$wl.log 2>&1 || exit $?
  echo "== $wl"; tail -1 gpurun_out/r4z_bench_$wl.log
done
timeout -k 10 400 python -u bench.py --height 768 --width 768 --batch 16 --steps 3 --warmup 1 \
  > gpurun_out/r4z_bench_sd21_768.log 2>&1 || exit $?
echo "== sd21 768"; tail -1 gpurun_out/r4z_bench_sd21_768.log
