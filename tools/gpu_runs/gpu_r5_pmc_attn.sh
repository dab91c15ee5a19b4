#!/bin/bash
# Round 5: PMC pass over the attention lab (flash64x2 vs the 128-query DMA kernel, flash2): MFMA / VALU issue.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn5 -o run --output-format csv -- \
  ./tools/gemm_lab/bin/attn_lab > gpurun_out/pmc_attn5.log 2>&1 || { tail -5 gpurun_out/pmc_attn5.log; exit 1; }
f=$(find gpurun_out/pmc_attn5 -name '*counter_collection.csv' | head -1)
python3 tools/gemm_lab/pmc_summary.py "$f" > gpurun_out/pmc_attn5.md
grep -i "flash\|attn" gpurun_out/pmc_attn5.md | cut -c1-300
