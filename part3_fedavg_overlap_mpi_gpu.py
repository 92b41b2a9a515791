#!/usr/bin/env python3
"""FedAvg ECG training entry point (API/CLI-compatible with the reference
Module_3/TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py).

Launch one process per MI355X (RCCL over xGMI):
    torchrun --standalone --nproc-per-node 8 part3_fedavg_overlap_mpi_gpu.py --data-root data/shards \
        --batch-size 256 --rounds 5 --local-steps 50 --config both --max-windows 20000
``mpiexec -n 8`` / ``srun`` also work (launcher env shim).  On a CPU box the same command runs with gloo.
New flags: --kernel-backend {auto,fused,torch} --amp-dtype {bf16,fp16,none} --overlap {none,tail,delayed}
--sync {fedavg,none,ddp} --no-bcast-every-round --ckpt-every N --resume --drop-prob p
--synthetic-windows N --labels {zeros,parity} --config-file cfg.yaml
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.config import FedAvgConfig, add_dataclass_args, from_args  # noqa: E402
from crossscale_ecg.parallel.env import init_distributed, shutdown_distributed, setup_device  # noqa: E402,F401
from crossscale_ecg.parallel.fedavg import broadcast_model, fedavg_allreduce, Communicator  # noqa: E402,F401
from crossscale_ecg.train.steps import train_step_G0, train_step_G1  # noqa: E402,F401
from crossscale_ecg.train.fedavg import run_fedavg, set_basic_seeds  # noqa: E402,F401
from crossscale_ecg.utils.csvio import append_results, RoundStats  # noqa: E402,F401


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    add_dataclass_args(ap, FedAvgConfig)
    ap.add_argument("--config-file", dest="config_file", default=None, help="YAML overrides")
    return ap


def main(argv=None):
    ns = build_parser().parse_args(argv)
    cfg = from_args(FedAvgConfig, ns)
    if cfg.config not in ("G0", "G1", "both"):
        raise SystemExit("--config must be G0, G1 or both")
    ctx = init_distributed()
    try:
        return run_fedavg(cfg, ctx)
    finally:
        shutdown_distributed()


if __name__ == "__main__":
    main()
