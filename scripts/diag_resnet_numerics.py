#!/usr/bin/env python3
"""ResNet1D engine gradient numerics: per-tensor relative error of the native engine against (a) the
bf16-emulating fp64 reference (models/resnet1d_ref.py), (b) plain fp64, and of torch bf16 autocast vs fp64."""
from __future__ import annotations

import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.resnet1d import resnet1d18, resnet1d34  # noqa: E402
from crossscale_ecg.models.resnet1d_ref import reference_grads  # noqa: E402
from crossscale_ecg.ops.resnet_engine import ResNetStepEngine  # noqa: E402


def rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def main():
    dev = torch.device("cuda:0")
    for depth, B in ((18, 32), (34, 32), (18, 128), (34, 128)):
        torch.manual_seed(0)
        m = (resnet1d18 if depth == 18 else resnet1d34)().to(dev)
        ref = copy.deepcopy(m)
        x = torch.randn(B, 1, 500, device=dev)
        y = torch.randint(0, 2, (B,), device=dev)
        eng = ResNetStepEngine(m, B, 500, use_graph=False)
        eng.set_batch(x, y)
        eng.forward_backward()
        torch.cuda.synchronize()
        grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
        _, gq = reference_grads(ref, x, y)
        r64 = copy.deepcopy(ref).double()
        F.cross_entropy(r64(x.double()), y).backward()
        g64 = {n: p.grad for n, p in r64.named_parameters()}
        ram = copy.deepcopy(ref)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            F.cross_entropy(ram(x), y).backward()
        gam = {n: p.grad for n, p in ram.named_parameters()}
        rows = [(n, rel(grads[n], gq[n]), rel(grads[n], g64[n]), rel(gam[n], g64[n]), rel(gq[n], g64[n]))
                for n in grads]
        worst = sorted(rows, key=lambda r: -r[1])[:6]
        med = lambda i: sorted(r[i] for r in rows)[len(rows) // 2]  # noqa: E731
        print(f"depth {depth} B {B}: engine-vs-emulated max {max(r[1] for r in rows):.4f} median {med(1):.4f} | "
              f"engine-vs-fp64 max {max(r[2] for r in rows):.4f} | autocast-vs-fp64 max {max(r[3] for r in rows):.4f}"
              f" | emulated-vs-fp64 max {max(r[4] for r in rows):.4f}")
        for n, a, b, c, d in worst:
            print(f"    {n:32s} eng/emu {a:.4f}  eng/fp64 {b:.4f}  amp/fp64 {c:.4f}  emu/fp64 {d:.4f}")
        eng.close()


if __name__ == "__main__":
    main()
