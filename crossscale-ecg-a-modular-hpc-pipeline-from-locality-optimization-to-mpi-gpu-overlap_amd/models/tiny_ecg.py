"""TinyECG: the 1-D CNN of the reference study.

Architecture and state_dict keys are identical to the reference
(Module_3/tiny_ecg_model.py:8-29, duplicated as ``Tiny1D`` in Module_1/bench_locality.py:8-21):

    Conv1d(1,16,k7,p3) -> ReLU -> Conv1d(16,16,k5,p2) -> ReLU -> AdaptiveAvgPool1d(1) -> Linear(16,C)

1,458 parameters for C=2 in 6 tensors: net.0.weight[16,1,7], net.0.bias[16], net.2.weight[16,16,5],
net.2.bias[16], head.weight[C,16], head.bias[C].

MI355X additions:
  * ``flatten_parameters()`` re-points every parameter into ONE contiguous fp32 buffer (in
    ``parameters()`` order).  The fused HIP train step reads/writes that buffer directly and FedAvg
    reduces it with a single RCCL call, while ``state_dict()``/``load_state_dict()`` keep working.
  * ``param_layout(C)`` gives the (offset, numel) table the HIP kernels are compiled against.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Tuple

import torch
import torch.nn as nn

C_HID = 16
K1, P1 = 7, 3
K2, P2 = 5, 2


def param_layout(num_classes: int = 2) -> "OrderedDict[str, Tuple[int, Tuple[int, ...]]]":
    """Flat fp32 layout: name -> (offset, shape). Order == ``TinyECG.parameters()``."""
    shapes = [
        ("net.0.weight", (C_HID, 1, K1)),
        ("net.0.bias", (C_HID,)),
        ("net.2.weight", (C_HID, C_HID, K2)),
        ("net.2.bias", (C_HID,)),
        ("head.weight", (num_classes, C_HID)),
        ("head.bias", (num_classes,)),
    ]
    out: "OrderedDict[str, Tuple[int, Tuple[int, ...]]]" = OrderedDict()
    off = 0
    for name, shp in shapes:
        n = 1
        for s in shp:
            n *= s
        out[name] = (off, shp)
        off += n
    return out


def num_params(num_classes: int = 2) -> int:
    lay = param_layout(num_classes)
    name, (off, shp) = next(reversed(lay.items()))
    n = 1
    for s in shp:
        n *= s
    return off + n


class TinyECG(nn.Module):
    """Very small 1D CNN for ECG windows. Input [B, 1, L] -> logits [B, num_classes]."""

    def __init__(self, num_classes: int = 2):
        super().__init__()
        self.num_classes = num_classes
        self.net = nn.Sequential(
            nn.Conv1d(1, C_HID, kernel_size=K1, padding=P1),
            nn.ReLU(inplace=True),
            nn.Conv1d(C_HID, C_HID, kernel_size=K2, padding=P2),
            nn.ReLU(inplace=True),
            nn.AdaptiveAvgPool1d(1),
        )
        self.head = nn.Linear(C_HID, num_classes)
        self._flat: torch.Tensor | None = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.net(x)
        x = x.squeeze(-1)
        return self.head(x)

    # ---------------------------------------------------------------- flat parameter storage
    @property
    def flat(self) -> torch.Tensor | None:
        return self._flat

    def flatten_parameters(self, pad_to: int = 64) -> torch.Tensor:
        """Move all parameters into one contiguous fp32 buffer (padded to ``pad_to`` elements)."""
        params = list(self.parameters())
        dev = params[0].device
        total = sum(p.numel() for p in params)
        padded = (total + pad_to - 1) // pad_to * pad_to
        flat = torch.zeros(padded, dtype=torch.float32, device=dev)
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                flat[off:off + n].copy_(p.detach().reshape(-1).float())
                p.data = flat[off:off + n].view_as(p)
                off += n
        self._flat = flat
        return flat

    def flat_grad_views(self, flat_grad: torch.Tensor) -> None:
        """Make each ``p.grad`` a view into ``flat_grad`` (same layout as the flat params)."""
        off = 0
        for p in self.parameters():
            n = p.numel()
            p.grad = flat_grad[off:off + n].view_as(p)
            off += n

    def _apply(self, fn, *args, **kwargs):  # keep the flat buffer coherent across .to()/.cuda()
        had_flat = self._flat is not None
        out = super()._apply(fn, *args, **kwargs)
        if had_flat:
            self._flat = None
            self.flatten_parameters()
        return out


def state_dict_to_flat(sd: Dict[str, torch.Tensor], num_classes: int = 2, pad_to: int = 64) -> torch.Tensor:
    lay = param_layout(num_classes)
    total = num_params(num_classes)
    flat = torch.zeros((total + pad_to - 1) // pad_to * pad_to, dtype=torch.float32)
    for name, (off, shp) in lay.items():
        t = sd[name].detach().float().reshape(-1).cpu()
        flat[off:off + t.numel()] = t
    return flat
