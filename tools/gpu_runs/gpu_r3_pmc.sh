#!/bin/bash
# Round-3 PMC passes (each counter set in its own run, hard-killed after 120 s): GEMM lab (SQ set: MFMA busy,
# waits, LDS) and attention lab (VALU / MFMA issue of flash64 vs flash2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PMC_SET=sq bash tools/gemm_lab/run_gpu.sh r3pmc > /dev/null || exit 1
cat gpurun_out/pmc_r3pmc.md | cut -c1-400
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn3 -o run --output-format csv -- \
  ./tools/gemm_lab/bin/attn_lab > gpurun_out/pmc_attn3.log 2>&1 || { tail -5 gpurun_out/pmc_attn3.log; exit 1; }
f=$(find gpurun_out/pmc_attn3 -name '*counter_collection.csv' | head -1)
python3 tools/gemm_lab/pmc_summary.py "$f" | tee gpurun_out/pmc_attn3.md | cut -c1-400
