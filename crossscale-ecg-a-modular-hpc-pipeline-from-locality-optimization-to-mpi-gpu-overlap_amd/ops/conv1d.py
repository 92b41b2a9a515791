"""Single-channel valid conv1d (the Module-2 op) on three backends, plus its HIP backward.

* ``hip``   - ``conv1d_batch_hip`` (csrc/kernels/conv1d_valid.hip), fp32 or bf16, async on the torch stream;
              ``blocking=True`` uses ``conv1d_batch_hip_flag`` (returns when the output is complete, like the
              reference's CPU kernel: the kernel's last workgroup publishes completion to a host-mapped word the
              caller polls) - the single-call path the Module-2 ``time_once`` metric measures.
              ``conv1d_valid_fn`` is the differentiable version (HIP dgrad + deterministic two-pass wgrad).
* ``cpu``   - ``conv1d_batch_omp_simd`` (csrc/cpu/conv1d_cpu.cpp), the reference C ABI
              (Module_2/conv1d_openmp_simd.c:21-28) with OpenMP + AVX2/AVX-512.
* ``torch`` - ``F.conv1d`` (MIOpen on the GPU / oneDNN on the CPU) — the baseline the paper compares to
              (Module_2/benchmark_part_2.py:75-82).

``run_omp_conv(x_np, w_np, nthreads)`` keeps the reference helper's signature (benchmark_part_2.py:48-59).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib
from ..utils import usable_cpus


def _as_2d(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 3:
        if x.shape[1] != 1:
            raise ValueError("conv1d_valid is single-channel: expected [B,1,L]")
        x = x[:, 0, :]
    if x.dim() != 2:
        raise ValueError(f"expected [B, L] or [B, 1, L], got {tuple(x.shape)}")
    return x.contiguous()


_HIP_FNS = {}  # dtype (or "sync") -> bound C function (after the first call)
_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _conv1d_hip_fast(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None,
                     blocking: bool = False) -> torch.Tensor | None:
    """Per-call fast path of the hip backend (the Module-2 benchmark times single calls, so Python overhead is
    part of the measured number, as the torch side's dispatch is part of its): no intermediate tensors, one
    raw-stream query.  Returns None when the operands need the general path (conversions, copies, checks)."""
    d = x.dim()
    if (_raw_stream is None or not x.is_cuda or not x.is_contiguous() or (d == 3 and x.shape[1] != 1)
            or d not in (2, 3) or w.dtype != torch.float32 or not w.is_contiguous() or w.device != x.device):
        return None
    if not _HIP_FNS:
        lib = _lib.kernels()  # raises if the HIP library is missing: no silent fallback on a GPU tensor
        _HIP_FNS.update({torch.float32: lib.conv1d_batch_hip, torch.bfloat16: lib.conv1d_batch_hip_bf16,
                         "sync": lib.conv1d_batch_hip_flag})
    fn = _HIP_FNS.get("sync" if blocking and x.dtype == torch.float32 else x.dtype)
    if fn is None:
        return None
    B, L, K = x.shape[0], x.shape[-1], w.numel()
    outL = L - K + 1
    if K < 1 or outL < 1:
        return None
    if out is None:
        out = torch.empty((B, 1, outL) if d == 3 else (B, outL), dtype=x.dtype, device=x.device)
    elif out.dtype != x.dtype or out.numel() != B * outL or not out.is_contiguous() or out.device != x.device:
        return None
    st = fn(x.data_ptr(), w.data_ptr(), out.data_ptr(), B, L, K, _raw_stream(x.device.index))
    if st:
        _lib.check(st, "conv1d_batch_hip")
    if blocking and x.dtype != torch.float32:
        torch.cuda.current_stream(x.device).synchronize()
    return out if out.dim() == d else out.view((B, 1, outL) if d == 3 else (B, outL))


class HipConv1dValid:
    """A bound single-channel valid conv1d on the HIP kernel - the op-object counterpart of ``nn.Conv1d(1, 1, K)``
    (taps held by the object, like the module holds its weight).  ``y = op(x, out)`` for x [B, L] / [B, 1, L]
    fp32 on the taps' device, out [B, L-K+1].  ``blocking``: return when y is complete (the reference CPU
    kernel's call semantics, Module_2/conv1d_openmp_simd.c:21-61): one native call that launches the kernel and
    polls a host-mapped word its last workgroup writes once every output store has drained (9.4-9.6 us at
    B=256, K=7 vs 14.0 for launch + hipStreamSynchronize, 16.7 polling hipStreamQuery; profiles/r2/
    conv1d_flag_call_ab.txt); else async on the current stream.  Per call it only re-checks the shapes
    and takes the data pointers."""

    def __init__(self, w: torch.Tensor, blocking: bool = True):
        if not w.is_cuda:
            raise ValueError("HipConv1dValid needs the taps on a GPU")
        self.w = w.detach().reshape(-1).to(torch.float32).contiguous()
        self.K = self.w.numel()
        lib = _lib.kernels()
        self._fn = lib.conv1d_batch_hip_flag if blocking else lib.conv1d_batch_hip
        self._wp = self.w.data_ptr()
        self._dev = self.w.device.index
        self._shapes = None

    def __call__(self, x: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        shapes = (x.shape, out.shape, x.dtype, out.dtype)
        if shapes != self._shapes:
            B, L = x.shape[0], x.shape[-1]
            if (x.dtype != torch.float32 or out.dtype != torch.float32 or not x.is_contiguous()
                    or not out.is_contiguous() or x.numel() != B * L or out.numel() != B * (L - self.K + 1)
                    or x.device != self.w.device or out.device != self.w.device):
                raise ValueError("HipConv1dValid: x must be contiguous fp32 [B, L] and out [B, L-K+1] on the "
                                 "taps' device")
            self._shapes, self._BL = shapes, (B, L)
        B, L = self._BL
        st = self._fn(x.data_ptr(), self._wp, out.data_ptr(), B, L, self.K, _raw_stream(self._dev))
        if st:
            _lib.check(st, "conv1d_batch_hip")
        return out


def conv1d_valid(x: torch.Tensor, w: torch.Tensor, backend: str = "auto", out: torch.Tensor | None = None,
                 nthreads: int | None = None, blocking: bool = False) -> torch.Tensor:
    """y[b, i] = sum_k x[b, i+k] w[k] for x [B, L] (or [B,1,L]), w [K] -> y [B, L-K+1] (same rank as x).

    ``blocking`` (hip): return only when the output is complete (one native launch + stream wait)."""
    if backend == "hip" or (backend == "auto" and x.is_cuda):
        y = _conv1d_hip_fast(x, w, out, blocking)
        if y is not None:
            return y
    keep3 = x.dim() == 3
    x2 = _as_2d(x)
    w1 = w.reshape(-1).contiguous()
    B, L = x2.shape
    K = w1.numel()
    if K < 1 or K > L:
        raise ValueError(f"kernel size {K} incompatible with L={L}")
    outL = L - K + 1
    if backend == "auto":
        backend = "hip" if x2.is_cuda else "cpu"
    if backend == "torch":
        y = F.conv1d(x2.unsqueeze(1), w1.to(x2.dtype).view(1, 1, K))
        return y if keep3 else y[:, 0, :]
    if backend == "hip":
        if not x2.is_cuda:
            raise ValueError("hip backend needs a CUDA tensor")
        wf = w1.to(device=x2.device, dtype=torch.float32)
        if out is None:
            out = torch.empty((B, outL), dtype=x2.dtype, device=x2.device)
        lib = _lib.kernels()
        if x2.dtype == torch.float32:
            st = lib.conv1d_batch_hip(x2.data_ptr(), wf.data_ptr(), out.data_ptr(), B, L, K,
                                      _lib.stream_ptr(x2.device))
        elif x2.dtype == torch.bfloat16:
            st = lib.conv1d_batch_hip_bf16(x2.data_ptr(), wf.data_ptr(), out.data_ptr(), B, L, K,
                                           _lib.stream_ptr(x2.device))
        else:
            raise ValueError(f"unsupported dtype {x2.dtype}")
        _lib.check(st, "conv1d_batch_hip")
        if blocking:
            torch.cuda.current_stream(x2.device).synchronize()
        return out.unsqueeze(1) if keep3 else out
    if backend == "cpu":
        if x2.is_cuda or x2.dtype != torch.float32:
            raise ValueError("cpu backend needs a CPU float32 tensor")
        y = torch.from_numpy(run_omp_conv(x2.numpy(), w1.float().numpy(), nthreads))
        return y.unsqueeze(1) if keep3 else y
    raise ValueError(f"unknown backend {backend!r}")


def conv1d_valid_backward(x: torch.Tensor, w: torch.Tensor, dy: torch.Tensor, need_dx: bool = True,
                          need_dw: bool = True):
    """HIP backward of ``conv1d_valid``: (dx [B, L] in x's dtype, dw [K] fp32) from dy [B, L-K+1]."""
    x2, dy2 = _as_2d(x), _as_2d(dy).to(x.dtype).contiguous()
    w1 = w.reshape(-1).to(device=x2.device, dtype=torch.float32).contiguous()
    B, L = x2.shape
    K = w1.numel()
    if dy2.shape != (B, L - K + 1):
        raise ValueError(f"dy must be [{B}, {L - K + 1}], got {tuple(dy2.shape)}")
    bf = x2.dtype == torch.bfloat16
    if x2.dtype not in (torch.float32, torch.bfloat16) or not x2.is_cuda:
        raise ValueError("conv1d_valid_backward needs a CUDA fp32/bf16 tensor")
    lib = _lib.kernels()
    stream = _lib.stream_ptr(x2.device)
    dx = dw = None
    if need_dx:
        dx = torch.empty_like(x2)
        fn = lib.conv1d_valid_dgrad_hip_bf16 if bf else lib.conv1d_valid_dgrad_hip
        _lib.check(fn(dy2.data_ptr(), w1.data_ptr(), dx.data_ptr(), B, L, K, stream), "conv1d_valid_dgrad_hip")
    if need_dw:
        n = int(lib.conv1d_valid_wgrad_ws_floats(B, L, K))
        ws = torch.empty(n, dtype=torch.float32, device=x2.device)
        dw = torch.empty(K, dtype=torch.float32, device=x2.device)
        fn = lib.conv1d_valid_wgrad_hip_bf16 if bf else lib.conv1d_valid_wgrad_hip
        _lib.check(fn(x2.data_ptr(), dy2.data_ptr(), dw.data_ptr(), ws.data_ptr(), n, B, L, K, stream),
                   "conv1d_valid_wgrad_hip")
    return dx, dw


class _Conv1dValidFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return conv1d_valid(x, w.detach().reshape(-1).float(), backend="hip")

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx, dw = conv1d_valid_backward(x, w, dy, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        if dx is not None and x.dim() == 3:
            dx = dx.unsqueeze(1)
        return dx, (dw.view_as(w).to(w.dtype) if dw is not None else None)


def conv1d_valid_fn(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Differentiable single-channel valid conv1d on the HIP kernels (forward, dgrad, wgrad)."""
    return _Conv1dValidFn.apply(x, w)


def run_omp_conv(x_np: np.ndarray, w_np: np.ndarray, nthreads: int | None = None,
                 y_np: np.ndarray | None = None) -> np.ndarray:
    """Native CPU kernel with the reference C ABI. x [B, L] float32, w [K] float32 -> y [B, L-K+1]."""
    x_np = np.ascontiguousarray(x_np, dtype=np.float32)
    w_np = np.ascontiguousarray(w_np, dtype=np.float32).reshape(-1)
    batch, L = x_np.shape
    K = w_np.shape[0]
    if K < 1 or K > L:
        raise ValueError(f"kernel size {K} incompatible with L={L}")
    outL = L - K + 1
    if y_np is None:
        y_np = np.empty((batch, outL), dtype=np.float32)
    elif y_np.shape != (batch, outL) or y_np.dtype != np.float32 or not y_np.flags.c_contiguous:
        raise ValueError("bad output buffer")
    fp = C.POINTER(C.c_float)
    _lib.cpu_lib().conv1d_batch_omp_simd(x_np.ctypes.data_as(fp), w_np.ctypes.data_as(fp), y_np.ctypes.data_as(fp),
                                        batch, L, K, int(nthreads or usable_cpus()))
    return y_np


def conv1d_valid_reference(x: np.ndarray, w: np.ndarray) -> np.ndarray:
    """float64 numpy reference (np.correlate per row)."""
    x = np.asarray(x, dtype=np.float64)
    w = np.asarray(w, dtype=np.float64).reshape(-1)
    return np.stack([np.correlate(r, w, mode="valid") for r in x])
