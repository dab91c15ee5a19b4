#!/bin/bash
# Round-6 closing check on the final tree: GPU test suite, smoke(), then bench lines (SD2.1 default config x2,
# Mistral b64, Flux 512^2 / 1024^2, ViT b32, mllama).  Each step has its own time limit; the first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  > gpurun_out/r6f_pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r6f_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f_smoke.log 2>&1 \
  || { tail -5 gpurun_out/r6f_smoke.log; exit 1; }
tail -1 gpurun_out/r6f_smoke.log
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 900 python -u bench.py "$@" > gpurun_out/r6f_$name.log 2>&1 || { tail -5 gpurun_out/r6f_$name.log; return 1; }
  echo "$name: $(grep '^{' gpurun_out/r6f_$name.log | tail -1 | cut -c1-420)"
}
run sd21_a --steps 10 --warmup 2 || exit 1
run mistral --workload mistral || exit 1
run flux512 --workload flux || exit 1
run flux1024 --workload flux --height 1024 --width 1024 || exit 1
run vit --workload vit || exit 1
run mllama --workload mllama || exit 1
run sd21_b --steps 10 --warmup 2 || exit 1
