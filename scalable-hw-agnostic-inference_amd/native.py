"""Loader for the in-tree native libraries built by ``csrc/build.py``.

GPU code paths call :func:`ops` which loads ``_native/libshai_kernels.so`` and
returns ``torch.ops.shai``.  If the library is missing or fails to load while a
GPU tensor needs it, we raise -- there is deliberately no silent eager fallback
for GPU tensors.  CPU tensors use the fp32 torch references in
``shai_amd.ops.reference`` (tests, and the CPU BERT "plumbing" config).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

# SHAI_KERNEL_DEBUG=1: the device debug flavour (``python csrc/build.py --debug``: bounds asserts + hazard-safe waits)
DEBUG = os.environ.get("SHAI_KERNEL_DEBUG", "0") == "1"
_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_native_debug" if DEBUG else "_native")
KERNELS_LIB = os.path.join(_DIR, "libshai_kernels.so")
RUNTIME_LIB = os.path.join(_DIR, "libshai_runtime.so")
COMM_LIB = os.path.join(_DIR, "libshai_comm.so")

_lock = threading.Lock()
_kernels_loaded = False
_kernels_error: Exception | None = None
_runtime = None
_comm = None


class NativeUnavailable(RuntimeError):
    pass


def _load_kernels() -> None:
    global _kernels_loaded, _kernels_error
    with _lock:
        if _kernels_loaded or _kernels_error is not None:
            return
        try:
            if not os.path.exists(KERNELS_LIB):
                raise NativeUnavailable(f"{KERNELS_LIB} not found; run `python csrc/build.py`")
            torch.ops.load_library(KERNELS_LIB)
            _kernels_loaded = True
            _autoload_tuning()
        except Exception as e:  # pragma: no cover - depends on build state
            _kernels_error = e


DEFAULT_TUNE_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "config",
                                 "gemm_tuning_mi355x.json")


def _autoload_tuning() -> None:
    """Pre-load GEMM tile/split-K choices measured on MI355X (config/gemm_tuning_mi355x.json, or
    ``SHAI_GEMM_TUNE_FILE``; "none" disables) so serving warm-up skips the per-shape autotune sweep.
    Shapes missing from the file are still autotuned on first use."""
    path = os.environ.get("SHAI_GEMM_TUNE_FILE", DEFAULT_TUNE_FILE)
    if path and path != "none" and os.path.exists(path):
        load_gemm_tuning(path)


def save_gemm_tuning(path: str) -> int:
    """Persist the GEMM autotuner cache (shape key -> tile config, split-K)."""
    import json
    entries = list(ops().gemm_tuning_export())
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(entries, f, indent=0)
    return len(entries)


def load_gemm_tuning(path: str) -> int:
    import json
    with open(path) as f:
        entries = json.load(f)
    return int(torch.ops.shai.gemm_tuning_import(entries))


def kernels_available() -> bool:
    _load_kernels()
    return _kernels_loaded


def ops():
    """Return ``torch.ops.shai``; raise loudly if the HIP kernels are not loadable."""
    _load_kernels()
    if not _kernels_loaded:
        raise NativeUnavailable(f"shai HIP kernels unavailable: {_kernels_error!r}")
    return torch.ops.shai


def runtime() -> ctypes.CDLL:
    """Host C++ runtime (block manager / scheduler), C ABI via ctypes."""
    global _runtime
    with _lock:
        if _runtime is None:
            if not os.path.exists(RUNTIME_LIB):
                raise NativeUnavailable(f"{RUNTIME_LIB} not found; run `python csrc/build.py`")
            _runtime = ctypes.CDLL(RUNTIME_LIB)
    return _runtime


def runtime_available() -> bool:
    try:
        runtime()
        return True
    except Exception:
        return False


def comm() -> ctypes.CDLL:
    """xGMI peer-to-peer all-reduce library (needs torch's HIP runtime loaded first)."""
    global _comm
    with _lock:
        if _comm is None:
            if not os.path.exists(COMM_LIB):
                raise NativeUnavailable(f"{COMM_LIB} not found; run `python csrc/build.py`")
            import torch.cuda  # noqa: F401  ensure torch's libamdhip64 is the one resolved
            _comm = ctypes.CDLL(COMM_LIB, mode=ctypes.RTLD_GLOBAL)
    return _comm


def loaded_libraries() -> list[str]:
    """Native .so files of this package mapped into the current process."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if _DIR in line:
                    p = line.split()[-1]
                    if p not in out:
                        out.append(p)
    except OSError:
        pass
    return out
