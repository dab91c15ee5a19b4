"""Device debug flavour: ``python csrc/build.py --debug`` compiles every kernel with
-DSHAI_KERNEL_DEBUG into ``_native_debug/`` (loaded when SHAI_KERNEL_DEBUG=1).  Here (CPU, hipcc cross-compiles
gfx950) the flag must turn the SHAI_DASSERT bounds checks of the hand-scheduled kernels into device asserts and
compile them away in the production flavour."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _device_asm(src, debug, tmp):
    out = os.path.join(tmp, ("dbg_" if debug else "rel_") + os.path.basename(src) + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + os.path.join(ROOT, "csrc"),
           "--cuda-device-only", "-S", src, "-o", out]
    if debug:
        cmd.insert(1, "-DSHAI_KERNEL_DEBUG")
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    with open(out) as f:
        return f.read()


@pytest.mark.skipif(shutil.which(HIPCC) is None and not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("src", ["csrc/comm/p2p_allreduce.hip", "csrc/kernels/conv_halo.hip"])
def test_debug_flavour_compiles_asserts_in(src, tmp_path):
    path = os.path.join(ROOT, src)
    dbg = _device_asm(path, True, str(tmp_path))
    rel = _device_asm(path, False, str(tmp_path))
    # a failing SHAI_DASSERT calls the device assert handler; production code has no such call
    assert "__assert_fail" in dbg or "assert" in dbg.lower()
    assert "__assert_fail" not in rel


def test_build_script_has_debug_flavour():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    import build
    assert build.OUT_DEBUG.endswith("_native_debug") and build.BUILD_DEBUG != build.BUILD
    import inspect
    assert "debug" in inspect.signature(build.build).parameters
