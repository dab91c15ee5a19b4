#!/bin/bash
# Round 3: wide GEMM epilogue in production.  GPU test suite (numerics of every forced tile config), the
# GEMM lab A/B with the no-drain persistent variant, then the driver's SD2.1 bench line and smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3w_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3w_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3w_pytest_gpu.log
bash tools/gemm_lab/run_gpu.sh wide2 > /dev/null || exit 1
python3 - <<'PY'
import re
cur = None
for line in open("gpurun_out/lab_wide2.log"):
    if line.startswith("=="):
        cur = line.split()[1]; print("\n" + cur, end=": ")
    m = re.match(r"\s+(\S+)\s+([\d.]+) us\s+([\d.]+) TF/s", line)
    if m: print(f"{m.group(1)}={m.group(3)}", end=" ")
    if "MISMATCH" in line: print("\nMISMATCH", line)
print()
PY
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3w_smoke.log 2>&1 || { tail -20 gpurun_out/r3w_smoke.log; exit 1; }
tail -1 gpurun_out/r3w_smoke.log | cut -c1-200
timeout -k 10 500 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3w_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r3w_bench_sd21.log | cut -c1-400
timeout -k 10 400 python -u bench.py --workload mistral > gpurun_out/r3w_bench_mistral.log 2>&1 || exit $?
echo "== mistral"; tail -1 gpurun_out/r3w_bench_mistral.log | cut -c1-400
bash tools/rocprof.sh r3w_sd21 -- bench.py --steps 1 --warmup 1 --latency-runs 0 > /dev/null || exit 1
head -30 gpurun_out/rocprof_r3w_sd21.md
bash tools/rocprof.sh r3w_mistral -- bench.py --workload mistral --steps 1 --warmup 1 > /dev/null || exit 1
head -30 gpurun_out/rocprof_r3w_mistral.md
