#!/bin/bash
# Round 3: flash2 d64 M segment with immediate-offset fragment reads and -m through the MFMA; GPU suite,
# attention lab A/B (new vs previous M segment), GEMM lab (GLU shapes), SD2.1 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r3f_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3f_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3f_pytest_gpu.log
timeout -k 10 300 ./tools/gemm_lab/bin/attn_lab > gpurun_out/r3f_attn_lab.log 2>&1 || { tail -20 gpurun_out/r3f_attn_lab.log; exit 1; }
cat gpurun_out/r3f_attn_lab.log
bash tools/gemm_lab/run_gpu.sh glu1 > /dev/null || exit 1
python3 - <<'PY'
import re
for line in open("gpurun_out/lab_glu1.log"):
    if line.startswith("=="): print("\n" + line.split()[1], end=": ")
    m = re.match(r"\s+(\S+)\s+([\d.]+) us\s+([\d.]+) TF/s", line)
    if m: print(f"{m.group(1)}={m.group(3)}", end=" ")
    if "MISMATCH" in line: print("\nMISMATCH", line)
print()
PY
timeout -k 10 500 python -u bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/r3f_bench_sd21.log 2>&1 || exit $?
echo "== sd21"; tail -1 gpurun_out/r3f_bench_sd21.log | cut -c1-300
