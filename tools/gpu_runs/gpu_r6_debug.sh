#!/bin/bash
# Round 6: the GPU test suite once on the device debug flavour (python csrc/build.py --debug: SHAI_DASSERT bounds
# checks on DMA offsets / LDS indices / ring slots, hazard-safe waits) with every kernel launch serialised
# (AMD_SERIALIZE_KERNEL=3).  Needs _native_debug/ in the pushed tree (drop it from .gpurunignore for the call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SHAI_KERNEL_DEBUG=1 AMD_SERIALIZE_KERNEL=3 timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf \
  --timeout 300 --timeout-method thread > gpurun_out/r6_debug_suite.log 2>&1
rc=$?
tail -5 gpurun_out/r6_debug_suite.log
exit $rc
