#!/bin/bash
# Round 4: decode attention grid A/B on short contexts (Mistral b64): one workgroup per item (default at <= 8
# splits) vs the persistent walk (SHAI_DECODE_PERSIST=1); decode tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4l_pytest.log 2>&1 || { tail -30 gpurun_out/r4l_pytest.log; exit 1; }
tail -1 gpurun_out/r4l_pytest.log
for v in default 1 default 1; do
  if [ $v = default ]; then E=""; else E="SHAI_DECODE_PERSIST=1"; fi
  env $E timeout -k 10 300 python -u bench.py --workload mistral --steps 2 --warmup 1 > gpurun_out/r4l_mistral_$v.log 2>&1 || exit $?
  echo "mistral persist=$v: $(tail -1 gpurun_out/r4l_mistral_$v.log | cut -c1-120)"
done
