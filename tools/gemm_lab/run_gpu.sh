#!/bin/bash
# GEMM lab on the GPU box: timing pass, then (optional) one PMC pass over the same binary.
#   bash tools/gemm_lab/run_gpu.sh <tag> [lab args...]         e.g. run_gpu.sh r1 --quick --plain
# PMC_SET (env) picks the counter set; empty = no PMC pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 ./tools/gemm_lab/bin/gemm_lab "$@" > gpurun_out/lab_$TAG.log 2>&1
rc=$?
cat gpurun_out/lab_$TAG.log
[ $rc -eq 0 ] || exit $rc
case "$PMC_SET" in
  sq) CTRS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  mem) CTRS="SQ_WAVE_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" ;;
  *) exit 0 ;;
esac
timeout -s KILL 120 rocprofv3 --pmc $CTRS -d gpurun_out/pmc_$TAG -o run --output-format csv -- \
  ./tools/gemm_lab/bin/gemm_lab "$@" > gpurun_out/pmc_$TAG.log 2>&1 || { tail -5 gpurun_out/pmc_$TAG.log; exit 1; }
f=$(find gpurun_out/pmc_$TAG -name '*counter_collection.csv' | head -1)
python3 tools/gemm_lab/pmc_summary.py "$f" | tee gpurun_out/pmc_$TAG.md
