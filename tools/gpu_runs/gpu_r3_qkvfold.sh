#!/bin/bash
# QKV split-K fold inside the decode attention kernel: exactness tests, LLM GPU tests, Mistral b64 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_skinny_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "qkv_fold or fused_decode" > gpurun_out/qf_t1.log 2>&1 || { tail -40 gpurun_out/qf_t1.log; exit 1; }
tail -1 gpurun_out/qf_t1.log
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_varlen_gpu.py tests/test_mllama_gpu.py -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/qf_t2.log 2>&1 || { tail -40 gpurun_out/qf_t2.log; exit 1; }
tail -1 gpurun_out/qf_t2.log
for v in 1 0 1 0; do
  SHAI_QKV_FOLD_IN_ATTN=$v timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/qf_m$v.log 2>&1 || exit $?
  echo "fold_in_attn=$v $(tail -1 gpurun_out/qf_m$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_tpot_ms"])')"
done
