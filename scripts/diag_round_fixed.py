#!/usr/bin/env python3
"""Diagnostic: fixed vs per-step cost of one TinyECG round-graph replay (B=256, L=500, PF + gather path).

For n in (1, 2, 5, 10, 20, 50) the round's batches are staged, then ONE replay of the n-step graph is timed with
hipEvents (GPU span) and the host clock (launch -> synchronize); median of 15 repetitions.  A least-squares fit
time = a + b * n separates the per-round fixed cost a (graph launch, first-step LDS path) from the step cost b."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, L, N = 256, 500, 20000
    x = torch.randn(N, L, device=dev)
    y = torch.zeros(N, dtype=torch.long, device=dev)
    ns = (1, 2, 5, 10, 20, 50)
    if os.environ.get("DIAG_WAVES"):  # force the step kernel's wave count (8 or 16) before any graph is captured
        from crossscale_ecg.ops import _lib
        _lib.kernels().ecg_tiny_force_waves(int(os.environ["DIAG_WAVES"]))
    tr = FusedTinyTrainer(TinyECG().to(dev), x, y, B, 50, lr=1e-2, momentum=0.9, seed=0)
    tr.prepare(list(ns))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {}
    for n in ns:
        gs, ws = [], []
        for _ in range(15):
            tr.prepare_round(n)
            torch.cuda.synchronize()
            e0.record()
            t0 = time.perf_counter()
            tr.launch_round(n)
            e1.record()
            torch.cuda.synchronize()
            ws.append((time.perf_counter() - t0) * 1e6)
            gs.append(e0.elapsed_time(e1) * 1e3)
        res[n] = (statistics.median(gs), statistics.median(ws))
        print(f"n={n:3d}: gpu {res[n][0]:8.1f} us  wall {res[n][1]:8.1f} us  ({res[n][0] / n:.2f} / {res[n][1] / n:.2f} per step)")
    for k, name in ((0, "gpu"), (1, "wall")):
        xs = list(ns)
        ys = [res[n][k] for n in ns]
        mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
        b = sum((a - mx) * (c - my) for a, c in zip(xs, ys)) / sum((a - mx) ** 2 for a in xs)
        print(f"fit {name}: fixed {my - b * mx:7.1f} us + {b:.3f} us/step")
    tr.close()


if __name__ == "__main__":
    main()
