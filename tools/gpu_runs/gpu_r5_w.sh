#!/bin/bash
# Round 5: flash2 built with VGPR-form MFMAs -- attention / Flux / LLM GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_flux_gpu.py tests/test_models_gpu.py tests/test_varlen_gpu.py tests/test_mllama_gpu.py -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/r5w_pytest.log 2>&1 || { tail -30 gpurun_out/r5w_pytest.log; exit 1; }
tail -1 gpurun_out/r5w_pytest.log
