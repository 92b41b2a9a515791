"""ctypes bindings for the in-tree native libraries (built by ``csrc/build.py``).

The HIP kernels are exposed through a plain C ABI (launchers take raw device pointers and the
``hipStream_t`` of the current torch stream), so no torch C++ headers are compiled and the same
symbols serve Python, C++ tools and graph capture.  ``torch`` is imported first so that the HIP
runtime torch ships (SONAME libamdhip64.so.7) is the one our libraries bind to.

Failure policy: on a machine with a GPU the HIP library MUST load - ``kernels()`` raises loudly if it
is missing (no silent eager fallback).  On CPU-only machines callers check ``kernels_available()``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must be loaded before libamdhip64 is resolved by our libraries)

LIB_DIR = os.environ.get("ECG_LIB_DIR") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")

_lock = threading.Lock()
_libs = {}

vp, i32, i64, f32 = C.c_void_p, C.c_int, C.c_long, C.c_float
f64p = C.POINTER(C.c_double)
i32p = C.POINTER(C.c_int)
i64p = C.POINTER(C.c_int64)

STATUS = {0: "ok", 1: "bad argument", 2: "problem too large for the fused kernel", 3: "HIP runtime error",
          4: "I/O error", 5: "timeout", 6: "end of data"}


class NativeError(RuntimeError):
    pass


def check(status: int, what: str) -> None:
    if status != 0:
        raise NativeError(f"{what} failed: status {status} ({STATUS.get(status, '?')})")


def _load(name: str) -> Optional[C.CDLL]:
    with _lock:
        if name in _libs:
            return _libs[name]
        path = os.path.join(LIB_DIR, name)
        lib = None
        if os.path.exists(path):
            lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
        _libs[name] = lib
        return lib


def _sig(lib, name, argtypes, restype=i32):
    fn = getattr(lib, name)
    fn.argtypes = argtypes
    fn.restype = restype
    return fn


def _bind_kernels(lib: C.CDLL) -> None:
    _sig(lib, "ecg_tiny_param_count", [i32])
    _sig(lib, "ecg_tiny_smem_bytes", [i32, i32])
    _sig(lib, "ecg_tiny_step_grads", [vp, i32, i64, vp, vp, vp, i32, vp, i32, i32, f32, i32, vp, vp])
    _sig(lib, "ecg_tiny_forward", [vp, i32, i64, vp, vp, i32, vp, i32, i32, vp, vp])
    _sig(lib, "ecg_tiny_wprep_bytes", [])
    _sig(lib, "ecg_tiny_train_step_pf", [vp, i32, i64, vp, vp, vp, vp, i32, vp, i32, i32, vp, f32, f32, f32, i32,
                                         vp, i32, vp])
    _sig(lib, "ecg_tiny_train_steps_pf", [vp, i32, i64, vp, vp, vp, vp, i32, vp, i32, i32, i32, vp, f32, f32, f32,
                                          i32, vp, i32, vp])
    _sig(lib, "ecg_tiny_prep", [vp, vp, vp])
    _sig(lib, "ecg_slab_reduce_sgd", [vp, i32, i32, i32, vp, vp, vp, vp, f32, f32, f32, i32, i32, vp, vp])
    _sig(lib, "ecg_tiny_train_step", [vp, i32, i64, vp, vp, vp, vp, i32, vp, i32, i32, vp, f32, f32, f32, i32,
                                      i32, vp, vp])
    _sig(lib, "ecg_round_graph_create", [C.POINTER(vp), vp, i32, i64, vp, vp, vp, vp, i32, vp, i32, i32, i32, vp,
                                         f32, f32, f32, i32, i32, vp, vp])
    _sig(lib, "ecg_round_graph_create_pf", [C.POINTER(vp), vp, i32, i64, vp, vp, vp, vp, i32, vp, i32, i32, i32,
                                            vp, f32, f32, f32, i32, vp, i32, i32, vp, vp])
    _sig(lib, "ecg_tiny_gather_floats", [i32, i32], i64)
    _sig(lib, "ecg_tiny_step_grads_twice", [vp, i32, i64, vp, vp, vp, i32, vp, i32, i32, f32, i32, vp, vp])
    _sig(lib, "ecg_tiny_force_waves", [i32])
    _sig(lib, "ecg_tiny_set_stamps", [vp])
    _sig(lib, "ecg_round_graph_launch", [vp, vp])
    _sig(lib, "ecg_round_graph_destroy", [vp])
    _sig(lib, "ecg_round_graph_upload", [vp, vp])
    _sig(lib, "conv1d_batch_hip", [vp, vp, vp, i32, i32, i32, vp])
    _sig(lib, "conv1d_batch_hip_sync", [vp, vp, vp, i32, i32, i32, vp])
    _sig(lib, "conv1d_batch_hip_spin", [vp, vp, vp, i32, i32, i32, vp])
    _sig(lib, "conv1d_batch_hip_flag", [vp, vp, vp, i32, i32, i32, vp])
    _sig(lib, "conv1d_valid_dgrad_hip", [vp, vp, vp, i32, i32, i32, vp])
    _sig(lib, "conv1d_valid_dgrad_hip_bf16", [vp, vp, vp, i32, i32, i32, vp])
    _sig(lib, "conv1d_valid_wgrad_ws_floats", [i32, i32, i32], i64)
    _sig(lib, "conv1d_valid_wgrad_hip", [vp, vp, vp, vp, i64, i32, i32, i32, vp])
    _sig(lib, "conv1d_valid_wgrad_hip_bf16", [vp, vp, vp, vp, i64, i32, i32, i32, vp])
    _sig(lib, "conv1d_batch_hip_bf16", [vp, vp, vp, i32, i32, i32, vp])
    _sig(lib, "ecg_sgd_flat", [vp, vp, vp, i64, f32, f32, f32, f32, i32, i32, f32, vp, vp])
    _sig(lib, "ecg_gather_rows_f32", [vp, i64, i32, vp, i32, vp, i64, i32, f32, vp])
    _sig(lib, "ecg_gather_rows_bf16", [vp, i64, i32, vp, i32, vp, i64, i32, f32, vp])
    for extra in ("_bind_conv_mc",):
        fn = globals().get(extra)
        if fn:
            fn(lib)


def kernels_available() -> bool:
    return _load("libecg_kernels.so") is not None


_kernels_lib: Optional[C.CDLL] = None


def kernels() -> C.CDLL:
    """The HIP kernel library (raises if it was not built)."""
    global _kernels_lib
    if _kernels_lib is not None:  # bound once; no lock on the per-launch path
        return _kernels_lib
    lib = _load("libecg_kernels.so")
    if lib is None:
        raise NativeError(f"libecg_kernels.so not found in {LIB_DIR}: run `python csrc/build.py` "
                          "(or __graft_entry__.build())")
    if not getattr(lib, "_ecg_bound", False):
        _bind_kernels(lib)
        lib._ecg_bound = True
    _kernels_lib = lib
    return lib


def io_lib() -> C.CDLL:
    lib = _load("libecg_io.so")
    if lib is None:
        raise NativeError(f"libecg_io.so not found in {LIB_DIR}: run `python csrc/build.py`")
    if not getattr(lib, "_ecg_bound", False):
        _sig(lib, "ecg_shard_open", [C.c_char_p, C.POINTER(vp), i64p, i64p])
        _sig(lib, "ecg_shard_data", [vp], vp)
        _sig(lib, "ecg_shard_close", [vp])
        _sig(lib, "ecg_prefetch_create", [C.POINTER(C.c_char_p), i32, i32, i32, i32, i32, i32, C.POINTER(vp), i64p])
        _sig(lib, "ecg_prefetch_start", [vp])
        _sig(lib, "ecg_prefetch_slot_ptr", [vp, i32], vp)
        _sig(lib, "ecg_prefetch_next", [vp, i32, i32p, i32p, f64p])
        _sig(lib, "ecg_prefetch_recycle", [vp, i32])
        _sig(lib, "ecg_prefetch_recycle_after", [vp, i32, vp])
        _sig(lib, "ecg_prefetch_h2d", [vp, i32, i32, vp, vp])
        _sig(lib, "ecg_prefetch_shutdown", [vp])
        _sig(lib, "ecg_prefetch_destroy", [vp])
        _sig(lib, "ecg_prefetch_error", [vp], C.c_char_p)
        _sig(lib, "ecg_upload_shards", [C.POINTER(C.c_char_p), i32, C.c_int64, C.c_int64, vp, C.c_int64, vp, i64p])
        _sig(lib, "ecg_upload_shards_mt", [C.POINTER(C.c_char_p), i32, C.c_int64, C.c_int64, vp, C.c_int64, i32, vp,
                                           i64p])
        lib._ecg_bound = True
    return lib


def io_available() -> bool:
    return _load("libecg_io.so") is not None


def cpu_lib() -> C.CDLL:
    lib = _load("libconv1d_cpu.so")
    if lib is None:
        raise NativeError(f"libconv1d_cpu.so not found in {LIB_DIR}: run `python csrc/build.py`")
    if not getattr(lib, "_ecg_bound", False):
        _sig(lib, "conv1d_batch_omp_simd", [vp, vp, vp, i32, i32, i32, i32], None)
        _sig(lib, "conv1d_cpu_isa", [])
        _sig(lib, "conv1d_cpu_set_isa", [i32])
        lib._ecg_bound = True
    return lib


def cpu_available() -> bool:
    return _load("libconv1d_cpu.so") is not None


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """Raw hipStream_t of torch's current stream on ``device`` (one C++ call: this sits on the launch path of
    every timed round, where building a torch Stream object first cost microseconds)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def loaded_library_paths() -> list:
    return [os.path.join(LIB_DIR, n) for n, lib in _libs.items() if lib is not None]
