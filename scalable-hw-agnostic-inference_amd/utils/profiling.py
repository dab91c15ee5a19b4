"""Tracing / profiling hooks.

The reference has no tracing in code (operators watch ``nvidia-smi`` / ``neuron-top``,
`mistral/README.md:41-55`); here every engine entry point is wrapped in a named range:

* ``range_("unet_step")`` pushes a ROCTx range (``libroctx64``) so ``rocprofv3 --marker-trace``
  groups the hand-written kernels under the engine phase that launched them, and a
  ``torch.profiler.record_function`` range for the PyTorch profiler.  Both are no-ops
  unless tracing is enabled, so the hot path pays one bool check.
* ``SHAI_PROFILE=1`` turns the ranges on; ``SHAI_PROFILE_DIR=<dir>`` additionally runs
  ``torch.profiler`` around each ``profile_session(...)`` block (the engine's generate / step)
  and writes a Chrome trace per session.
* ``tools/rocprof.sh`` is the kernel-level counterpart (``rocprofv3 --kernel-trace --stats``).

Ranges are NOT emitted inside HIP-graph capture (graph replay has no host ranges anyway).
"""
from __future__ import annotations

import contextlib
import ctypes
import itertools
import os
import time
from typing import Optional

_ENABLED = os.environ.get("SHAI_PROFILE", "0") not in ("", "0", "false", "False")
_DIR = os.environ.get("SHAI_PROFILE_DIR", "")
_roctx = None
_session_id = itertools.count()


def enabled() -> bool:
    return _ENABLED


def enable(flag: bool = True, trace_dir: Optional[str] = None) -> None:
    """Programmatic switch (tests, bench --profile)."""
    global _ENABLED, _DIR
    _ENABLED = bool(flag)
    if trace_dir is not None:
        _DIR = trace_dir


def _lib():
    global _roctx
    if _roctx is None:
        _roctx = False
        for name in ("libroctx64.so", "libroctx64.so.4", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                break
            except (OSError, AttributeError):
                continue
    return _roctx or None


def _capturing() -> bool:
    try:
        import torch
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    except Exception:
        return False


@contextlib.contextmanager
def range_(name: str):
    """Named ROCTx + torch.profiler range (no-op unless SHAI_PROFILE=1)."""
    if not _ENABLED or _capturing():
        yield
        return
    import torch
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    if _ENABLED and (lib := _lib()) is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def profile_session(name: str):
    """torch.profiler session around one engine call when SHAI_PROFILE_DIR is set; writes
    ``<dir>/<name>-<pid>-<n>.json`` (Chrome trace).  Otherwise just a named range."""
    if not (_ENABLED and _DIR) or _capturing():
        with range_(name):
            yield
        return
    import torch
    from torch.profiler import ProfilerActivity, profile
    os.makedirs(_DIR, exist_ok=True)
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts, record_shapes=False) as prof:
        with range_(name):
            yield
    path = os.path.join(_DIR, f"{name}-{os.getpid()}-{next(_session_id)}.json")
    prof.export_chrome_trace(path)


class StepTimer:
    """Wall-clock per named phase (host side; synchronises only when ``sync=True``)."""

    def __init__(self, sync: bool = False):
        self.sync = sync
        self.totals: dict = {}
        self.counts: dict = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.sync:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
        t0 = time.perf_counter()
        try:
            with range_(name):
                yield
        finally:
            if self.sync:
                import torch
                if torch.cuda.is_available():
                    torch.cuda.synchronize()
            self.totals[name] = self.totals.get(name, 0.0) + time.perf_counter() - t0
            self.counts[name] = self.counts.get(name, 0) + 1

    def report(self) -> dict:
        return {k: {"total_ms": round(v * 1e3, 3), "calls": self.counts[k]} for k, v in self.totals.items()}
