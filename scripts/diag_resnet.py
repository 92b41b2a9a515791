#!/usr/bin/env python3
"""ResNet1D numerics diagnostic: per-parameter gradient error of the hip backend and of torch bf16 autocast, both
against the fp32 torch model (same weights, same batch)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.resnet1d import resnet1d18  # noqa: E402


def grads(m, x, y, amp=False):
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        loss = F.cross_entropy(m(x), y)
    loss.backward()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}, loss.item()


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.manual_seed(0)
    m = resnet1d18(backend="torch").cuda()
    x = torch.randn(B, 1, 500, device="cuda")
    y = torch.randint(0, 2, (B,), device="cuda")
    g32, l32 = grads(m, x, y)
    gam, lam = grads(m, x, y, amp=True)
    m.backend = "hip"
    ghp, lhp = grads(m, x, y)
    print(f"loss fp32 {l32:.5f} amp {lam:.5f} hip {lhp:.5f}")
    for n in g32:
        print(f"{n:32s} amp {rel(gam[n], g32[n]):.4f} hip {rel(ghp[n], g32[n]):.4f} hip-vs-amp {rel(ghp[n], gam[n]):.4f}")
