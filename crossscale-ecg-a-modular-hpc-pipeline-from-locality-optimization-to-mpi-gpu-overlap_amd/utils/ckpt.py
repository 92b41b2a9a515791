"""Checkpoint / resume (not present in the reference: SURVEY §5.4).

Layout (plain ``torch.save``, loaded with ``weights_only=True`` - no pickle execution):

* ``checkpoints/fedavg_{cfg}_round{r:05d}.pt`` - written by rank 0: ``{"round", "config", "model"
  (TinyECG state_dict keys), "momentum" (rank 0's), "rng_cpu", "args"}``.  ``TinyECG.load_state_dict`` works on
  its ``"model"`` entry anywhere.
* ``checkpoints/fedavg_{cfg}_round{r:05d}.rank{k}.pt`` - written by EVERY rank into its own ``ckpt_dir``: the
  client-local state FedAvg never averages (SGD momentum, the batch sampler's generator / epoch block / cursor,
  the CPU RNG) and, for ``--sync none`` (independent clients), the client's own flat weights.
* ``--overlap delayed``: a checkpoint of round r holds avg_r (the all-reduce of round r's weights, waited for on
  the device); the run itself keeps its one-round-stale correction pending, so its trajectory does not depend
  on ``--ckpt-every``.  A resume starts from avg_r with nothing in flight: resuming ends the staleness once.

Resume (``train.fedavg.run_fedavg``): rank 0 alone resolves the latest round (its directory is the only one
guaranteed to hold the model file - no shared filesystem is assumed), broadcasts the round index, loads the
weights and broadcasts them over RCCL; every rank then restores its own client state if its directory has
the matching ``.rank{k}.pt`` file (otherwise momentum restarts at zero and the sampler from its seed).
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


def rank_state_path(ckpt_dir: str, round_idx: int, config: str, rank: int) -> str:
    return ckpt_path(ckpt_dir, round_idx, config)[:-3] + f".rank{rank}.pt"


def _atomic_save(state, path: str) -> str:
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)  # atomic: a crash mid-write never leaves a truncated checkpoint
    return path


def save_checkpoint(path: str, round_idx: int, model: torch.nn.Module, momentum: Optional[torch.Tensor] = None,
                    config: str = "", args: Optional[Dict[str, Any]] = None) -> str:
    state = {
        "round": int(round_idx),
        "config": config,
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "momentum": None if momentum is None else momentum.detach().cpu(),
        "rng_cpu": torch.get_rng_state(),
        "args": {k: (v if isinstance(v, (int, float, str, bool, type(None))) else str(v))
                 for k, v in (args or {}).items()},
    }
    return _atomic_save(state, path)


def trainer_local_state(trainer) -> Dict[str, Any]:
    """Client-local state of a trainer (FusedTinyTrainer / ResNetEngineTrainer / TorchLocalTrainer)."""
    st: Dict[str, Any] = {"rng_cpu": torch.get_rng_state()}
    mom = getattr(trainer, "mom", None)
    if isinstance(mom, torch.Tensor):
        st["momentum"] = mom.detach().cpu()
    opt = getattr(trainer, "opt", None)
    if opt is not None:
        bufs = [opt.state.get(p, {}).get("momentum_buffer") for g in opt.param_groups for p in g["params"]]
        st["momentum_list"] = [None if b is None else b.detach().cpu() for b in bufs]
    sampler = getattr(trainer, "sampler", None)
    if sampler is not None and hasattr(sampler, "state_dict"):
        st["sampler"] = sampler.state_dict()
    return st


def load_trainer_local_state(trainer, st: Dict[str, Any]) -> None:
    mom = getattr(trainer, "mom", None)
    if isinstance(mom, torch.Tensor) and st.get("momentum") is not None:
        if st["momentum"].shape != mom.shape:
            raise ValueError(f"momentum shape {tuple(st['momentum'].shape)} != {tuple(mom.shape)}")
        mom.copy_(st["momentum"].to(mom.device))
    opt = getattr(trainer, "opt", None)
    if opt is not None and st.get("momentum_list") is not None:
        params = [p for g in opt.param_groups for p in g["params"]]
        for p, b in zip(params, st["momentum_list"]):
            if b is not None:
                opt.state[p]["momentum_buffer"] = b.to(p.device).clone()
    sampler = getattr(trainer, "sampler", None)
    if sampler is not None and st.get("sampler") is not None:
        sampler.load_state_dict(st["sampler"])
    if st.get("rng_cpu") is not None:
        torch.set_rng_state(st["rng_cpu"])


def save_rank_state(ckpt_dir: str, round_idx: int, config: str, rank: int, trainer,
                    client_weights: Optional[torch.Tensor] = None) -> str:
    """``client_weights``: the client's own flat weights, for runs whose clients are never averaged
    (``--sync none``): a resumed independent client continues from them, not from rank 0's model."""
    st = trainer_local_state(trainer)
    if client_weights is not None:
        st["client_weights"] = client_weights.detach().cpu().clone()
    return _atomic_save(st, rank_state_path(ckpt_dir, round_idx, config, rank))


def load_checkpoint(path: str) -> Dict[str, Any]:
    return torch.load(path, map_location="cpu", weights_only=True)


def latest_checkpoint(ckpt_dir: str, config: str = "") -> Optional[str]:
    tag = f"{config}_" if config else ""
    paths = [p for p in glob.glob(os.path.join(ckpt_dir, f"fedavg_{tag}round*.pt"))
             if re.search(r"round(\d+)\.pt$", p)]
    if not paths:
        return None
    return max(paths, key=lambda p: int(re.search(r"round(\d+)\.pt$", p).group(1)))
