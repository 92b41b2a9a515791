"""Workload configuration: one dataclass per workload, populated from argparse with the reference's flag
names and defaults, plus the MI355X flags.  ``--config file.yaml`` overrides defaults
(yaml.safe_load only)."""
from __future__ import annotations

import argparse
from dataclasses import dataclass, field, fields
from typing import List, Optional


@dataclass
class FedAvgConfig:
    # ---- reference flags (TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:140-147) ----
    data_root: Optional[str] = None
    batch_size: int = 256
    rounds: int = 10
    local_steps: int = 50
    max_windows: int = 30000
    config: str = "both"  # G0 | G1 | both
    # ---- MI355X additions ----
    kernel_backend: str = "auto"  # auto | fused | hip | torch  (hip = MFMA conv kernels for ResNet1D)
    amp_dtype: str = "bf16"  # bf16 | fp16 | none  (dtype of the G1 configuration)
    overlap: str = "none"  # none | tail (exact, ResNet engine) | delayed (stale-by-one)
    sync: str = "fedavg"  # fedavg | none | ddp
    bcast_every_round: bool = True  # the reference broadcasts every round; RCCL AVG makes it redundant
    synthetic_windows: int = 0  # >0: skip shards, generate N(0,1) windows on device
    labels: str = "zeros"  # zeros (reference) | parity (learnable)
    win_len: int = 500
    lr: float = 1e-2
    momentum: float = 0.9
    seed: int = 1234
    drop_prob: float = 0.0  # FL client dropout injection (weighted FedAvg, zero-weight skip)
    # latency injection: host sleep inside each round's weight-independent batch preparation (the work that
    # --overlap tail places under the in-flight all-reduce); lets the overlap tests prove exposure < comm
    inject_prep_delay_ms: float = 0.0
    bucket_mb: float = 4.0  # ResNet1D tail / DDP gradient-bucket size (~1-4 MB per collective)
    ckpt_every: int = 0
    ckpt_dir: str = "checkpoints"
    resume: bool = False
    results_csv: str = "results/fedavg_results.csv"
    jsonl: Optional[str] = None
    model: str = "tiny_ecg"
    num_classes: int = 2
    quiet: bool = False


@dataclass
class PseudoFLConfig:
    # ---- reference flags (Module_3/part3_mpi_gpu_train.py:424-430) ----
    batch_size: int = 256
    steps: int = 200
    max_windows: int = 20000
    data_root: Optional[str] = None
    # ---- MI355X additions ----
    kernel_backend: str = "auto"
    amp_dtype: str = "bf16"
    loader: str = "gpu"  # gpu (GPU-resident shards, reference active path) | stream (pinned + copy-stream H2D)
    synthetic_windows: int = 0
    win_len: int = 500
    seed: int = 1234
    results_csv: str = "results/part3_mpi_cuda_results.csv"
    quiet: bool = False


def add_dataclass_args(ap: argparse.ArgumentParser, cls, skip: List[str] = ()) -> None:
    for f in fields(cls):
        if f.name in skip:
            continue
        flag = "--" + f.name.replace("_", "-")
        default = f.default
        if f.type in ("bool", bool):
            ap.add_argument(flag, action=argparse.BooleanOptionalAction, default=default)
        else:
            typ = {"int": int, "float": float, "str": str}.get(str(f.type).replace("Optional[", "").rstrip("]"), str)
            ap.add_argument(flag, type=typ, default=default)


def from_args(cls, ns: argparse.Namespace):
    kw = {f.name: getattr(ns, f.name) for f in fields(cls) if hasattr(ns, f.name)}
    cfg = cls(**kw)
    path = getattr(ns, "config_file", None)
    if path:
        import yaml
        with open(path) as fh:
            over = yaml.safe_load(fh) or {}
        for k, v in over.items():
            if hasattr(cfg, k):
                setattr(cfg, k, v)
    return cfg
