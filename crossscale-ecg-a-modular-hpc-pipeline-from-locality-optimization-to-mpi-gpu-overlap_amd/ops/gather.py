"""Batch gather (+ optional per-window z-score) into a preallocated batch buffer.

HIP kernel ``ecg_gather_rows_{f32,bf16}`` (csrc/kernels/gather_batch.hip) replaces the reference's
``x_gpu[sel]`` index kernel (Module_3/shard_dataset.py:133-136) and the CPU-side z-score of the LABL
prefetcher (Module_1/labl_loader(EXPERIMENTAL).py:65-69).  Writing into ``out`` keeps addresses static
so the gather can live inside a captured graph.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib


def gather_rows(x: torch.Tensor, idx: Optional[torch.Tensor], batch: Optional[int] = None,
                out: Optional[torch.Tensor] = None, normalize: bool = False, eps: float = 1e-8,
                dtype: torch.dtype = torch.float32) -> torch.Tensor:
    """out[b] = x[idx[b]] (z-scored per window if ``normalize``), out is [B, L] in ``dtype``."""
    if x.dim() != 2 or x.dtype != torch.float32 or x.stride(1) != 1:
        raise ValueError("x must be float32 [N, L] with unit inner stride")
    B = batch if batch is not None else (idx.numel() if idx is not None else x.shape[0])
    L = x.shape[1]
    if idx is not None and (idx.dtype != torch.int32 or idx.numel() < B or not idx.is_contiguous()):
        raise ValueError("idx must be contiguous int32 with >= B entries")
    if not x.is_cuda:
        rows = x[idx[:B].long()] if idx is not None else x[:B]
        if normalize:
            m = rows.double().mean(1, keepdim=True)
            s = rows.double().std(1, unbiased=False, keepdim=True) + eps
            rows = ((rows.double() - m) / s).float()
        res = rows.to(dtype)
        if out is not None:
            out.copy_(res)
            return out
        return res
    if out is None:
        out = torch.empty((B, L), dtype=dtype, device=x.device)
    if out.shape[0] < B or out.shape[1] != L or out.stride(1) != 1:
        raise ValueError("bad output buffer")
    lib = _lib.kernels()
    fn = lib.ecg_gather_rows_f32 if out.dtype == torch.float32 else lib.ecg_gather_rows_bf16
    if out.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError(f"unsupported output dtype {out.dtype}")
    st = fn(x.data_ptr(), x.stride(0), L, _lib.ptr(idx), B, out.data_ptr(), out.stride(0), int(normalize), eps,
            _lib.stream_ptr(x.device))
    _lib.check(st, "ecg_gather_rows")
    return out
