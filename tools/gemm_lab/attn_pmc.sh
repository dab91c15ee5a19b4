set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn -o run --output-format csv -- python3 tools/bench_kernels.py --only attn > gpurun_out/pmc_attn.log 2>&1 || { tail -5 gpurun_out/pmc_attn.log; exit 1; }
f=$(find gpurun_out/pmc_attn -name '*counter_collection.csv' | head -1)
python3 tools/gemm_lab/pmc_summary.py "$f" | grep -E "flash|kernel [|]" | tee gpurun_out/pmc_attn.md
grep "op=attn" gpurun_out/pmc_attn.log
