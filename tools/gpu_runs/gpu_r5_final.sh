#!/bin/bash
# Round-5 closing check on the final tree: build() from scratch on the box (./build is not uploaded), the GPU suite,
# smoke, the SD2.1 bench line, and every workload's bench line for the README table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( time timeout -k 10 900 python -u -c "import __graft_entry__ as g; g.build()" ) > gpurun_out/r5z_build.log 2>&1 || { tail -30 gpurun_out/r5z_build.log; exit 1; }
grep "native build" gpurun_out/r5z_build.log | cut -c1-200; grep real gpurun_out/r5z_build.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r5z_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r5z_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r5z_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5z_smoke.log 2>&1 || { tail -20 gpurun_out/r5z_smoke.log; exit 1; }
tail -1 gpurun_out/r5z_smoke.log | cut -c1-200
run() {  # name, bench args
  local name=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/r5z_$name.log 2>&1 || { tail -20 gpurun_out/r5z_$name.log; return 1; }
  echo "$name: $(grep '^{' gpurun_out/r5z_$name.log | tail -1 | cut -c1-400)"
}
run sd21 --steps 8 --warmup 2 || exit 1
run mistral --workload mistral --steps 2 --warmup 1 || exit 1
run flux512 --workload flux --steps 3 --warmup 1 --inference-steps 10 || exit 1
run flux1024 --workload flux --height 1024 --width 1024 --steps 2 --warmup 1 --inference-steps 10 || exit 1
run vit --workload vit --steps 50 --warmup 5 || exit 1
run t5 --workload t5 --steps 20 --warmup 3 || exit 1
run mllama --workload mllama --steps 2 --warmup 1 || exit 1
