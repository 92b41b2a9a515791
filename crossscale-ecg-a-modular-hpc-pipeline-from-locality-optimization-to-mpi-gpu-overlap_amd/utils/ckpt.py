"""Checkpoint / resume (not present in the reference: SURVEY §5.4).

Layout: ``checkpoints/fedavg_round{r:05d}.pt`` written by rank 0 with plain ``torch.save`` of
``{"round", "config", "model" (TinyECG state_dict keys), "momentum" (flat, rank 0), "rng", "args"}``.
``load_checkpoint`` uses ``weights_only=True`` (no pickle execution).  On resume rank 0 loads and the
weights are broadcast over RCCL so every client starts the next round from identical weights.
"""
from __future__ import annotations

import glob
import os
import re
from typing import Any, Dict, Optional

import torch


def ckpt_path(ckpt_dir: str, round_idx: int, config: str = "") -> str:
    tag = f"{config}_" if config else ""
    return os.path.join(ckpt_dir, f"fedavg_{tag}round{round_idx:05d}.pt")


def save_checkpoint(path: str, round_idx: int, model: torch.nn.Module, momentum: Optional[torch.Tensor] = None,
                    config: str = "", args: Optional[Dict[str, Any]] = None) -> str:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    state = {
        "round": int(round_idx),
        "config": config,
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "momentum": None if momentum is None else momentum.detach().cpu(),
        "rng_cpu": torch.get_rng_state(),
        "args": {k: (v if isinstance(v, (int, float, str, bool, type(None))) else str(v))
                 for k, v in (args or {}).items()},
    }
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)  # atomic: a crash mid-write never leaves a truncated checkpoint
    return path


def load_checkpoint(path: str) -> Dict[str, Any]:
    return torch.load(path, map_location="cpu", weights_only=True)


def latest_checkpoint(ckpt_dir: str, config: str = "") -> Optional[str]:
    tag = f"{config}_" if config else ""
    paths = glob.glob(os.path.join(ckpt_dir, f"fedavg_{tag}round*.pt"))
    if not paths:
        return None
    return max(paths, key=lambda p: int(re.search(r"round(\d+)\.pt$", p).group(1)))
