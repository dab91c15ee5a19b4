#!/bin/bash
# Round 6: skinny kernel with the 16-B cross-wave reduction / epilogue -- decode GEMM tests, then re-race every
# decode-shaped (M <= 64) tuning entry (they were dropped from the cache: tools/gpu_runs/tune_nodecode.json) through
# the Mistral b64 / b32, mllama and ViT benches, then the Mistral b64 bench line on the re-raced cache.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_skinny_gpu.py tests/test_fp8_gpu.py tests/test_kernels_gpu.py -q -x \
  -k "skinny or decode or fp8 or splitk" --timeout 120 --timeout-method thread > gpurun_out/r6n_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r6n_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r6n_tests.log | head; exit $rc; }
cp tools/gpu_runs/tune_nodecode.json gpurun_out/tune_r6n.json
export SHAI_GEMM_TUNE_FILE=gpurun_out/tune_r6n.json SHAI_GEMM_TUNE_SAVE=gpurun_out/tune_r6n.json
for spec in "mistral64:--workload mistral --steps 1 --warmup 1 --batch 64" \
            "mistral32:--workload mistral --steps 1 --warmup 1 --batch 32" \
            "mllama:--workload mllama --steps 1 --warmup 1" \
            "vit:--workload vit --steps 2 --warmup 1"; do
  wl=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 python -u bench.py $args > gpurun_out/r6n_retune_$wl.log 2>&1 || { tail -5 gpurun_out/r6n_retune_$wl.log; exit 1; }
  echo "$wl: $(grep '^{' gpurun_out/r6n_retune_$wl.log | tail -1 | cut -c1-200)"
done
unset SHAI_GEMM_TUNE_SAVE
timeout -k 10 600 python -u bench.py --workload mistral > gpurun_out/r6n_mistral.log 2>&1 || { tail -5 gpurun_out/r6n_mistral.log; exit 1; }
echo "final: $(grep '^{' gpurun_out/r6n_mistral.log | tail -1 | cut -c1-300)"
