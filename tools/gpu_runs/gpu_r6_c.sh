#!/bin/bash
# Round 6: halo conv iteration -- numerics + kernel A/B at the SD2.1 shapes only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_halo_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r6c_halo_tests.log 2>&1 || { tail -40 gpurun_out/r6c_halo_tests.log; exit 1; }
tail -1 gpurun_out/r6c_halo_tests.log
timeout -k 10 400 python -u tools/bench_halo.py --out gpurun_out/r6c_halo_bench.json > gpurun_out/r6c_halo_bench.log 2>&1 \
  || { tail -20 gpurun_out/r6c_halo_bench.log; exit 1; }
python - <<'PY'
import json
for r in json.load(open("gpurun_out/r6c_halo_bench.json")):
    print(r["shape"], {k: v for k, v in r.items() if k.endswith("_us")})
PY
