#!/bin/bash
# Round 4: decode attention over a 128k context: contiguous vs scattered block tables, splits 16 / 32 / 64.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/bench_kernels.py --only dattn_long,dattn > gpurun_out/r4n_dattn.log 2>&1 || { tail -20 gpurun_out/r4n_dattn.log; exit 1; }
grep "decode_attn" gpurun_out/r4n_dattn.log
