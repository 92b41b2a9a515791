#!/usr/bin/env python3
"""Minimal driver for rocprofv3 PMC passes over the fused TinyECG gradient kernel and the slab reduction:
300 eager two-launch steps (B=256, L=500) after a warm-up."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    x = torch.randn(20000, 500, device=dev)
    y = torch.zeros(20000, dtype=torch.long, device=dev)
    torch.manual_seed(0)
    tr = FusedTinyTrainer(TinyECG().to(dev), x, y, 256, 50, seed=0, use_graph=False)
    for _ in range(6):
        tr.run_round(50)
    torch.cuda.synchronize()
    print("loss", tr.avg_loss())
    tr.close()


if __name__ == "__main__":
    main()
