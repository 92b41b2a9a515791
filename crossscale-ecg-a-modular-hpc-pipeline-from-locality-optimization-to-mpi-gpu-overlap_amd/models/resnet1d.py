"""ResNet1D-18/34 for ECG windows: the "scaling stress" model of BASELINE.json config 5 (not in the reference).

Standard 1-D ResNet: stem Conv1d(1,64,k7,s2,p3)+BN+ReLU+MaxPool(3,2,1), BasicBlock stages [3,4,6,3] (ResNet-34)
or [2,2,2,2] (ResNet-18) at widths 64/128/256/512 (first block of stages 2-4 strided), global average pool,
Linear(512, C).  Input [B, 1, L] -> logits [B, C].  ~7.2 M parameters (ResNet-34).

Backends (``model.backend``):
  * ``"torch"`` - nn.Conv1d / BatchNorm1d in NCL (MIOpen), usable under torch.autocast.
  * ``"hip"``   - channels-last (NLC) bf16 activations end-to-end through the stages; every 3-tap and 1x1
    conv runs on ``ops.conv_mc.conv1d_nlc`` (MFMA implicit GEMM fwd / dgrad / wgrad); BatchNorm runs as
    the same nn.BatchNorm1d modules on a [B*L, C] view (fp32 statistics).  The stem (C_in = 1) stays on
    MIOpen.  Parameters / state_dict keys are identical in both backends.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F


def _bn_nlc(bn: nn.BatchNorm1d, x: torch.Tensor) -> torch.Tensor:
    B, L, C = x.shape
    return bn(x.reshape(B * L, C).float()).view(B, L, C)


class BasicBlock1D(nn.Module):
    expansion = 1

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.conv1 = nn.Conv1d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm1d(cout)
        self.conv2 = nn.Conv1d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm1d(cout)
        self.downsample = None
        if stride != 1 or cin != cout:
            self.downsample = nn.Sequential(nn.Conv1d(cin, cout, 1, stride, bias=False), nn.BatchNorm1d(cout))

    def forward(self, x: torch.Tensor) -> torch.Tensor:  # NCL
        idt = x if self.downsample is None else self.downsample(x)
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + idt)

    def forward_nlc(self, x: torch.Tensor) -> torch.Tensor:  # NLC bf16
        from ..ops.conv_mc import conv1d_nlc
        if self.downsample is None:
            idt = x.float()
        else:
            c, bn = self.downsample[0], self.downsample[1]
            idt = _bn_nlc(bn, conv1d_nlc(x, c.weight, None, c.stride[0], 0))
        out = F.relu(_bn_nlc(self.bn1, conv1d_nlc(x, self.conv1.weight, None, self.conv1.stride[0], 1)))
        out = _bn_nlc(self.bn2, conv1d_nlc(out.to(torch.bfloat16), self.conv2.weight, None, 1, 1))
        return F.relu(out + idt).to(torch.bfloat16)


class ResNet1D(nn.Module):
    def __init__(self, layers: Sequence[int] = (3, 4, 6, 3), widths: Sequence[int] = (64, 128, 256, 512),
                 num_classes: int = 2, in_channels: int = 1, backend: str = "torch"):
        super().__init__()
        self.num_classes = num_classes
        self.backend = backend
        self.conv1 = nn.Conv1d(in_channels, widths[0], 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm1d(widths[0])
        self.maxpool = nn.MaxPool1d(3, 2, 1)
        stages: List[nn.Module] = []
        cin = widths[0]
        for i, (n, w) in enumerate(zip(layers, widths)):
            blocks = []
            for j in range(n):
                blocks.append(BasicBlock1D(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w
            stages.append(nn.Sequential(*blocks))
        self.layer1, self.layer2, self.layer3, self.layer4 = stages
        self.fc = nn.Linear(cin, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv1d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm1d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

        self._space = None

    # ---------------------------------------------------------------- flat parameter space (FedAvg / flat SGD)
    @property
    def flat(self):
        return None if self._space is None else self._space.flat

    def flatten_parameters(self, include_buffers: bool = True) -> torch.Tensor:
        """All parameters + BN running statistics as views into one fp32 buffer (parallel.flat.FlatParamSpace):
        FedAvg of the whole state is then a single RCCL all-reduce."""
        from ..parallel.flat import FlatParamSpace
        self._space = FlatParamSpace(self, include_buffers=include_buffers)
        return self._space.flat

    def _apply(self, fn, *args, **kwargs):
        had = self._space is not None
        out = super()._apply(fn, *args, **kwargs)
        if had:
            self._space = None
            self.flatten_parameters()
        return out

    def stem(self, x: torch.Tensor) -> torch.Tensor:
        return self.maxpool(F.relu(self.bn1(self.conv1(x))))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.stem(x)
        if self.backend == "hip" and x.is_cuda:
            h = x.transpose(1, 2).contiguous().to(torch.bfloat16)  # NCL -> NLC once
            for stage in (self.layer1, self.layer2, self.layer3, self.layer4):
                for blk in stage:
                    h = blk.forward_nlc(h)
            feat = h.float().mean(dim=1)
        else:
            for stage in (self.layer1, self.layer2, self.layer3, self.layer4):
                x = stage(x)
            feat = x.mean(dim=2)
        return self.fc(feat)


def resnet1d34(num_classes: int = 2, backend: str = "torch", **kw) -> ResNet1D:
    return ResNet1D((3, 4, 6, 3), num_classes=num_classes, backend=backend, **kw)


def resnet1d18(num_classes: int = 2, backend: str = "torch", **kw) -> ResNet1D:
    return ResNet1D((2, 2, 2, 2), num_classes=num_classes, backend=backend, **kw)
