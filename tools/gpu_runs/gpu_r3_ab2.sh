#!/bin/bash
# A/Bs on one box: flash2 d64 with / without the pre-scaled Q; Mistral b64 decode with the cold-tuned choices
# (A), o_proj / down on the in-kernel fixup (B), plus qkv on skinny2 (C); fp8 engine tests (W8A8 prefill) and
# the fp8 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for pre in 1 0; do
  SHAI_FLASH2_PRE=$pre timeout -k 10 300 python -u tools/bench_kernels.py --only attn > gpurun_out/r3_ab2_attn_$pre.log 2>&1 || { tail -20 gpurun_out/r3_ab2_attn_$pre.log; exit 1; }
  echo "== PRE=$pre"; grep "op=attn" gpurun_out/r3_ab2_attn_$pre.log | head -3
done
for v in A B C; do
  SHAI_GEMM_TUNE_FILE=config/ab/tune_$v.json timeout -k 10 300 python -u bench.py --workload mistral > gpurun_out/r3_ab2_m_$v.log 2>&1 || { tail -20 gpurun_out/r3_ab2_m_$v.log; exit 1; }
  echo "== mistral $v"; tail -1 gpurun_out/r3_ab2_m_$v.log | cut -c1-200
done
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_ab2_fp8_tests.log 2>&1 || { tail -30 gpurun_out/r3_ab2_fp8_tests.log; exit 1; }
tail -1 gpurun_out/r3_ab2_fp8_tests.log
timeout -k 10 300 python -u bench.py --workload mistral --quantization fp8 > gpurun_out/r3_ab2_m_fp8.log 2>&1 || { tail -20 gpurun_out/r3_ab2_m_fp8.log; exit 1; }
echo "== mistral fp8"; tail -1 gpurun_out/r3_ab2_m_fp8.log | cut -c1-600
