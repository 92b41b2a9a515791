"""roctx ranges (visible in ``rocprofv3 --marker-trace`` / Perfetto) and an optional torch.profiler export.

The reference has no profiler integration.  ``range("comm")`` etc. bracket the data /
H2D / compute / comm phases; the ranges come from the ROCm roctx library through ctypes (the same
library torch ships), and become no-ops when it is unavailable.
"""
from __future__ import annotations

import ctypes
import os
from contextlib import contextmanager
from typing import Optional

_roctx = None
_tried = False


def _lib():
    global _roctx, _tried
    if _tried:
        return _roctx
    _tried = True
    import torch
    # rocprofv3 (rocprofiler-sdk) records the markers of its own roctx library; the legacy roctracer libroctx64
    # (also the copy torch ships) is only seen by the old tracer, so the SDK library comes first
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cands = [os.path.join(rocm, "lib", "librocprofiler-sdk-roctx.so"),
             os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"),
             os.path.join(rocm, "lib", "libroctx64.so")]
    for c in cands:
        if os.path.exists(c):
            try:
                lib = ctypes.CDLL(c)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _roctx = lib
                break
            except (OSError, AttributeError):
                continue
    return _roctx


ENABLED = os.environ.get("ECG_ROCTX", "1") != "0"


@contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    lib = _lib() if ENABLED else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def available() -> bool:
    return _lib() is not None


@contextmanager
def torch_profile(trace_path: Optional[str]):
    """Chrome-trace export via torch.profiler (ROCm/roctracer backed) when ``trace_path`` is set."""
    if not trace_path:
        yield None
        return
    import torch
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts) as prof:
        yield prof
    prof.export_chrome_trace(trace_path)
