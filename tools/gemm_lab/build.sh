#!/bin/bash
# Build the standalone GEMM lab (tools/gemm_lab/gemm_lab.cpp + the GEMM kernel sources) for gfx950.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/build/gemm_lab
mkdir -p "$OUT"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -I$ROOT/csrc -DSHAI_GEMM_LAB"
for src in gemm_lds gemm_8ph gemm_w4 gemm_ws gemv attention attention2 attention3; do
  # incremental: rebuild an object only when its source or a shared header is newer
  if [ ! -f "$OUT/$src.o" ] || [ -n "$(find "$ROOT/csrc/kernels/$src.hip" "$ROOT/csrc/kernels/"*.h -newer "$OUT/$src.o")" ]; then
    extra=""
    { [ "$src" = gemm_w4 ] || [ "$src" = gemm_ws ]; } && extra="-mllvm -pragma-unroll-threshold=100000"
    [ "$src" = gemm_ws ] && extra="$extra -fno-slp-vectorize"   # as csrc/build.py EXTRA_KFLAGS
    { [ "$src" = attention3 ] || [ "$src" = attention2 ]; } && extra="-mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize"
    hipcc $FLAGS $extra -c "$ROOT/csrc/kernels/$src.hip" -o "$OUT/$src.o" &
  fi
done
hipcc $FLAGS -x hip -c "$ROOT/tools/gemm_lab/gemm_lab.cpp" -o "$OUT/gemm_lab.o" &
hipcc $FLAGS -x hip -c "$ROOT/tools/gemm_lab/attn_lab.cpp" -o "$OUT/attn_lab.o" &
wait
[ -s "$OUT/gemm_lab.o" ] && [ "$OUT/gemm_lab.o" -nt "$ROOT/tools/gemm_lab/gemm_lab.cpp" ] || { echo "gemm_lab.o stale"; exit 1; }
mkdir -p "$ROOT/tools/gemm_lab/bin"
hipcc --offload-arch=gfx950 "$OUT"/gemm_lab.o "$OUT"/gemm_lds.o "$OUT"/gemm_8ph.o "$OUT"/gemm_w4.o "$OUT"/gemm_ws.o "$OUT"/gemv.o \
  -o "$ROOT/tools/gemm_lab/bin/gemm_lab"
hipcc --offload-arch=gfx950 "$OUT"/attn_lab.o "$OUT"/attention.o "$OUT"/attention2.o "$OUT"/attention3.o -o "$ROOT/tools/gemm_lab/bin/attn_lab"
# G8_FLAGS="...": a second GEMM lab whose gemm_8ph.hip (v4) is built with extra compiler flags (A/B of codegen)
if [ -n "${G8_FLAGS:-}" ]; then
  hipcc $FLAGS -DSHAI_GEMM_LAB $G8_FLAGS -c "$ROOT/csrc/kernels/gemm_8ph.hip" -o "$OUT/gemm_8ph_x.o"
  hipcc --offload-arch=gfx950 "$OUT"/gemm_lab.o "$OUT"/gemm_lds.o "$OUT"/gemm_8ph_x.o "$OUT"/gemm_w4.o "$OUT"/gemm_ws.o "$OUT"/gemv.o \
    -o "$ROOT/tools/gemm_lab/bin/gemm_lab_x"
fi
# ATTN2_FLAGS="...": a second attention lab whose attention2.hip (flash2) is built with extra compiler flags (A/B of
# codegen; attention3.hip's flags came out of the same A/B)
if [ -n "${ATTN2_FLAGS:-}" ]; then
  hipcc $FLAGS $ATTN2_FLAGS -c "$ROOT/csrc/kernels/attention2.hip" -o "$OUT/attention2_x.o"
  hipcc --offload-arch=gfx950 "$OUT"/attn_lab.o "$OUT"/attention.o "$OUT"/attention2_x.o "$OUT"/attention3.o -o "$ROOT/tools/gemm_lab/bin/attn_lab_x"
fi
echo "built tools/gemm_lab/bin/gemm_lab tools/gemm_lab/bin/attn_lab"
