"""Eager PyTorch training steps (reference semantics, the ``--kernel-backend torch`` path).

* ``train_step_G0`` <- TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:103-114 (fp32, sync + loss.item())
* ``train_step_G1`` <- :117-132 (AMP).  The reference used fp16 ``torch.cuda.amp.autocast()`` +
  ``GradScaler``; on MI355X the default AMP dtype is bf16 (no scaler needed).  ``amp_dtype=torch.float16``
  keeps the scaler path for parity runs.
``sync=False`` drops the per-step device sync / ``.item()`` (the loss is returned as a device tensor).
"""
from __future__ import annotations

from typing import Optional, Union

import torch
import torch.nn.functional as F


def _sync(device: torch.device):
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def train_step_G0(model, x, y, opt, device, sync: bool = True) -> Union[float, torch.Tensor]:
    model.train()
    opt.zero_grad(set_to_none=True)
    logits = model(x)
    loss = F.cross_entropy(logits, y)
    loss.backward()
    opt.step()
    if not sync:
        return loss.detach()
    _sync(torch.device(device))
    return float(loss.item())


def train_step_G1(model, x, y, opt, scaler: Optional[torch.amp.GradScaler], device, amp_dtype=torch.bfloat16,
                  sync: bool = True) -> Union[float, torch.Tensor]:
    device = torch.device(device)
    model.train()
    opt.zero_grad(set_to_none=True)
    with torch.autocast(device_type=device.type, dtype=amp_dtype, enabled=device.type == "cuda" or
                        amp_dtype == torch.bfloat16):
        logits = model(x)
        loss = F.cross_entropy(logits, y)
    if scaler is not None and scaler.is_enabled():
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
    else:
        loss.backward()
        opt.step()
    if not sync:
        return loss.detach()
    _sync(device)
    return float(loss.item())


def make_scaler(device, amp_dtype) -> Optional[torch.amp.GradScaler]:
    device = torch.device(device)
    if amp_dtype == torch.float16 and device.type == "cuda":
        return torch.amp.GradScaler("cuda")
    return None
