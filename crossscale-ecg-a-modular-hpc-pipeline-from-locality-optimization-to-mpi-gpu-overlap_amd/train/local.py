"""Local (per-client) trainers.

``TorchLocalTrainer`` is the eager-PyTorch client (reference code path: per step ``next(batch_iter)``
device gather + fwd/CE/bwd/SGD, Module_3/TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:197-204), used for
``--kernel-backend torch``, for models without a fused kernel (ResNet1D) and as the CPU/gloo path.
It shares the ``run_steps`` / ``avg_loss`` interface of ``ops.fused_tiny.FusedTinyTrainer``.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from ..data.dataset import DeviceIndexSampler


class TorchLocalTrainer:
    def __init__(self, model: torch.nn.Module, x: torch.Tensor, y: torch.Tensor, batch_size: int,
                 lr: float = 1e-2, momentum: float = 0.9, weight_decay: float = 0.0,
                 amp_dtype: Optional[torch.dtype] = torch.bfloat16, seed: Optional[int] = None,
                 sync_each_step: bool = False):
        self.model, self.x, self.y, self.B = model, x, y, batch_size
        self.device = x.device
        self.opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=momentum, weight_decay=weight_decay)
        self.amp_dtype = amp_dtype
        self.scaler = torch.amp.GradScaler("cuda") if (amp_dtype == torch.float16 and x.is_cuda) else None
        self.sampler = DeviceIndexSampler(x.shape[0], batch_size, self.device, seed=seed)
        self._idx = torch.empty((1, batch_size), dtype=torch.int32, device=self.device)
        self.loss_acc = torch.zeros((), dtype=torch.float32, device=self.device)
        self._loss_steps = 0
        self.sync_each_step = sync_each_step
        self.steps_done = 0

    def step(self) -> torch.Tensor:
        self.sampler.fill(self._idx)
        sel = self._idx[0].long()
        xb, yb = self.x[sel].unsqueeze(1), self.y[sel]
        self.model.train()
        self.opt.zero_grad(set_to_none=True)
        use_amp = self.amp_dtype is not None and (self.device.type == "cuda" or self.amp_dtype == torch.bfloat16)
        with torch.autocast(device_type=self.device.type, dtype=self.amp_dtype or torch.float32, enabled=use_amp):
            loss = F.cross_entropy(self.model(xb), yb)
        if self.scaler is not None:
            self.scaler.scale(loss).backward()
            self.scaler.step(self.opt)
            self.scaler.update()
        else:
            loss.backward()
            self.opt.step()
        if self.sync_each_step and self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.steps_done += 1
        return loss.detach()

    def run_steps(self, n: int, reset_loss: bool = True) -> None:
        if reset_loss:
            self.loss_acc.zero_()
            self._loss_steps = 0
        for _ in range(n):
            self.loss_acc += self.step().float()
        self._loss_steps += n

    run_round = run_steps

    def prepare_round(self, n: int, reset_loss: bool = True) -> None:
        """Eager steps draw their batch inside ``step``; only the loss window is reset here."""
        if reset_loss:
            self.loss_acc.zero_()
            self._loss_steps = 0

    def launch_round(self, n: int, next_n=None) -> None:
        self.run_steps(n, reset_loss=False)

    def avg_loss(self) -> float:
        return float(self.loss_acc.item()) / max(1, self._loss_steps)

    def reset_momentum(self):
        for st in self.opt.state.values():
            if "momentum_buffer" in st and st["momentum_buffer"] is not None:
                st["momentum_buffer"].zero_()
