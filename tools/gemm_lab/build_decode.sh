#!/bin/bash
# Build the decode-GEMM lab (tools/gemm_lab/decode_lab.cpp + the GEMM kernel sources it links) for gfx950 into
# build/decode_lab/ (run on the GPU box: the binary is not shipped).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/build/decode_lab
mkdir -p "$OUT"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -I$ROOT/csrc -DSHAI_GEMM_LAB"
for src in gemm_lds gemm_8ph gemm_w4 gemm_ws gemv; do
  extra=""
  { [ "$src" = gemm_w4 ] || [ "$src" = gemm_ws ]; } && extra="-mllvm -pragma-unroll-threshold=100000"
  [ "$src" = gemm_ws ] && extra="$extra -fno-slp-vectorize"
  hipcc $FLAGS $extra -c "$ROOT/csrc/kernels/$src.hip" -o "$OUT/$src.o" &
done
hipcc $FLAGS -x hip -c "$ROOT/tools/gemm_lab/decode_lab.cpp" -o "$OUT/decode_lab.o" &
wait
hipcc --offload-arch=gfx950 "$OUT"/decode_lab.o "$OUT"/gemm_lds.o "$OUT"/gemm_8ph.o "$OUT"/gemm_w4.o "$OUT"/gemm_ws.o \
  "$OUT"/gemv.o -o "$OUT/decode_lab"
echo "built $OUT/decode_lab"
