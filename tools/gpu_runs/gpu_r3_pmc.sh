#!/bin/bash
# PMC counters of the decode gate_up GEMM (64 x 28672 x 4096, GLU + folded RMSNorm) per kernel variant; each
# counter pass is its own hard-killed run.  Kernel time from a kernel-trace run of the same driver.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum"
P2="FETCH_SIZE TCC_EA0_RDREQ_sum"
for cfg in 1201 1251 1000; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/kt_$cfg -o run --output-format csv -- python3 tools/pmc_decode_gemm.py $cfg > gpurun_out/pmc/kt_$cfg.log 2>&1 || { tail -5 gpurun_out/pmc/kt_$cfg.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $P1 -d gpurun_out/pmc/p1_$cfg -o run --output-format csv -- python3 tools/pmc_decode_gemm.py $cfg > gpurun_out/pmc/p1_$cfg.log 2>&1 || { tail -5 gpurun_out/pmc/p1_$cfg.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $P2 -d gpurun_out/pmc/p2_$cfg -o run --output-format csv -- python3 tools/pmc_decode_gemm.py $cfg > gpurun_out/pmc/p2_$cfg.log 2>&1 || { tail -5 gpurun_out/pmc/p2_$cfg.log; exit 1; }
  echo "== cfg $cfg done"
done
find gpurun_out/pmc -name '*kernel_trace.csv' -delete
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.md && cat gpurun_out/pmc/summary.md
