# 256x320 pipelined GEMM configs: numerics, then SD2.1 with a fresh autotune (all configs) saved to gpurun_out/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm3_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_g3.log 2>&1 || { tail -30 gpurun_out/pytest_g3.log; exit 1; }
tail -2 gpurun_out/pytest_g3.log
SHAI_GEMM_TUNE_FILE=none SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_sd_b32.json timeout -k 10 900 python -u bench.py --steps 2 > gpurun_out/bench_sd_fresh.log 2>&1 || { tail -5 gpurun_out/bench_sd_fresh.log; exit 1; }
tail -1 gpurun_out/bench_sd_fresh.log | cut -c1-200
python3 - <<'PY'
import json, collections
e = json.load(open("gpurun_out/tune_sd_b32.json"))
c = collections.Counter(x.split("=")[1].split(",")[0] for x in e)
print("cfg histogram", dict(c))
PY
