"""Flat-buffer SGD optimizer backed by ``ecg_sgd_flat`` (csrc/kernels/fused_sgd.hip).

Drop-in for ``torch.optim.SGD(params, lr, momentum, dampening, weight_decay, nesterov)`` when all
parameters live in one contiguous fp32 buffer (``TinyECG.flatten_parameters()`` or
``parallel.flat.FlatParamSpace``).  One launch updates every parameter; on CPU tensors it falls back to
the same math in torch (used by the gloo tests).  ``inv_scale``/``found_inf`` implement the fp16
GradScaler contract (unscale + skip on overflow) for the ``--amp-dtype fp16`` path.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib


class FlatSGD:
    def __init__(self, flat_params: torch.Tensor, flat_grads: torch.Tensor, lr: float = 1e-2, momentum: float = 0.0,
                 dampening: float = 0.0, weight_decay: float = 0.0, nesterov: bool = False):
        if flat_params.shape != flat_grads.shape or flat_params.dtype != torch.float32:
            raise ValueError("flat params/grads must be matching fp32 buffers")
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        self.p, self.g = flat_params, flat_grads
        self.lr, self.momentum, self.dampening, self.wd, self.nesterov = lr, momentum, dampening, weight_decay, nesterov
        self.buf = torch.zeros_like(flat_params) if momentum != 0 else None
        self.first = True

    def zero_grad(self):
        self.g.zero_()

    @torch.no_grad()
    def step(self, inv_scale: float = 1.0, found_inf: Optional[torch.Tensor] = None):
        if self.p.is_cuda:
            lib = _lib.kernels()
            st = lib.ecg_sgd_flat(self.p.data_ptr(), self.g.data_ptr(), _lib.ptr(self.buf), self.p.numel(), self.lr,
                                  self.momentum, self.dampening, self.wd, int(self.nesterov), int(self.first),
                                  inv_scale, _lib.ptr(found_inf), _lib.stream_ptr(self.p.device))
            _lib.check(st, "ecg_sgd_flat")
        else:
            g = self.g * inv_scale
            if found_inf is not None:
                bad = ~torch.isfinite(g).all()
                found_inf.fill_(int(bad))
                if bad:
                    return
            d = g + self.wd * self.p if self.wd else g
            if self.momentum != 0:
                if self.first:
                    self.buf.copy_(d)
                else:
                    self.buf.mul_(self.momentum).add_(d, alpha=1 - self.dampening)
                d = d + self.momentum * self.buf if self.nesterov else self.buf
            self.p.add_(d, alpha=-self.lr)
        self.first = False

    def state_dict(self):
        return {"lr": self.lr, "momentum": self.momentum, "dampening": self.dampening, "weight_decay": self.wd,
                "nesterov": self.nesterov, "first": self.first,
                "momentum_buffer": None if self.buf is None else self.buf.detach().cpu()}

    def load_state_dict(self, sd):
        self.first = bool(sd.get("first", False))
        if self.buf is not None and sd.get("momentum_buffer") is not None:
            self.buf.copy_(sd["momentum_buffer"].to(self.buf.device))
