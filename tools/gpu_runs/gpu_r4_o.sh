#!/bin/bash
# Round 4: rotated split slots in the persistent decode attention: decode tests, the 128k microbenchmark, the
# long-context lines and Mistral b64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( while sleep 60; do echo "running $(date +%T)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode" -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r4o_pytest.log 2>&1 || { tail -30 gpurun_out/r4o_pytest.log; exit 1; }
tail -1 gpurun_out/r4o_pytest.log
timeout -k 10 300 python -u tools/bench_kernels.py --only dattn_long > gpurun_out/r4o_dattn.log 2>&1 || { tail -20 gpurun_out/r4o_dattn.log; exit 1; }
grep "decode_attn" gpurun_out/r4o_dattn.log
for P in 65536 127744; do
  timeout -k 10 400 python -u -m shai_amd.bench.long_context --model llama31_8b --prompt-len $P --chunk 8192 \
    --background 16 --gen 128 > gpurun_out/r4o_long_$P.log 2>&1 || { tail -20 gpurun_out/r4o_long_$P.log; exit 1; }
  tail -1 gpurun_out/r4o_long_$P.log | cut -c1-400
done
timeout -k 10 300 python -u bench.py --workload mistral --steps 2 --warmup 1 > gpurun_out/r4o_mistral.log 2>&1 || exit $?
echo "mistral: $(tail -1 gpurun_out/r4o_mistral.log | cut -c1-120)"
