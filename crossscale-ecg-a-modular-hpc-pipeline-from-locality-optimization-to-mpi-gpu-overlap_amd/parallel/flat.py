"""Flat parameter space for arbitrary modules: every parameter (and, optionally, every floating-point buffer such
as BatchNorm running statistics) becomes a view into ONE contiguous fp32 device buffer.

Why: FedAvg / DDP over RCCL is then one ``all_reduce`` of one buffer per round (the reference's
``mpi_avg_params`` in part3_mpi_gpu_train.py does one ``MPI.Allreduce`` per tensor after a host copy), the flat
SGD kernel (ops.sgd.FlatSGD) updates all weights in one launch, and a checkpoint is one tensor.  The layout is
padded to 64 elements per segment so each view starts 256-byte aligned (one HBM burst / dwordx4 per lane).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch
import torch.nn as nn

ALIGN = 64


class FlatParamSpace:
    def __init__(self, module: nn.Module, include_buffers: bool = True, dtype: torch.dtype = torch.float32):
        self.module = module
        self.entries: List[Tuple[nn.Module, str, bool, int, torch.Size]] = []  # (owner, name, is_param, off, shape)
        off = 0
        for mod in module.modules():  # parameters first (module order) ...
            for name, p in mod._parameters.items():
                if p is None:
                    continue
                self.entries.append((mod, name, True, off, p.shape))
                off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.param_numel = off  # ... so the optimizer runs over flat[:param_numel] only
        if include_buffers:
            for mod in module.modules():
                for name, b in mod._buffers.items():
                    if b is None or not b.is_floating_point():
                        continue
                    self.entries.append((mod, name, False, off, b.shape))
                    off += (b.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        dev = next(iter(module.parameters())).device
        self.flat = torch.zeros(off, dtype=dtype, device=dev)
        with torch.no_grad():
            for mod, name, is_param, o, shp in self.entries:
                src = mod._parameters[name] if is_param else mod._buffers[name]
                n = src.numel()
                view = self.flat[o:o + n].view(shp)
                view.copy_(src.detach())
                if is_param:
                    src.data = view
                else:
                    mod._buffers[name] = view
        self.n_params = sum(e[4].numel() for e in self.entries if e[2])

    def grad_buffer(self) -> torch.Tensor:
        """A flat gradient buffer over the parameter segment; each ``p.grad`` becomes a view into it."""
        g = torch.zeros(self.param_numel, dtype=self.flat.dtype, device=self.flat.device)
        for mod, name, is_param, o, shp in self.entries:
            if is_param:
                p = mod._parameters[name]
                p.grad = g[o:o + p.numel()].view(shp)
        return g

    def param_mask(self) -> torch.Tensor:
        """1 where the flat element belongs to a parameter, 0 for buffers and padding."""
        m = torch.zeros_like(self.flat)
        for _, _, is_param, o, shp in self.entries:
            if is_param:
                m[o:o + shp.numel()] = 1
        return m

    def layout(self) -> Dict[str, Tuple[int, Tuple[int, ...]]]:
        names = {id(m): n for n, m in self.module.named_modules()}
        out = {}
        for mod, name, _, o, shp in self.entries:
            pre = names.get(id(mod), "")
            out[f"{pre}.{name}" if pre else name] = (o, tuple(shp))
        return out

    def offset_of(self, tensor: torch.Tensor) -> int:
        """Element offset of a parameter / buffer view inside the flat buffer."""
        return (tensor.data_ptr() - self.flat.data_ptr()) // self.flat.element_size()
