"""The in-tree native libraries must dlopen (all symbols resolved) -- catches e.g. kernel launch stubs a
host pass silently dropped, which otherwise only shows up as a load failure on the GPU box."""
import ctypes
import os

import pytest

from shai_amd import native


@pytest.mark.parametrize("lib", [native.KERNELS_LIB, native.RUNTIME_LIB, native.COMM_LIB])
def test_native_library_links(lib):
    if not os.path.exists(lib):
        pytest.skip(f"{lib} not built (python csrc/build.py)")
    if lib == native.COMM_LIB:
        import torch.cuda  # noqa: F401  (resolves libamdhip64 the way native.comm() does)
    ctypes.CDLL(lib, mode=ctypes.RTLD_GLOBAL)
