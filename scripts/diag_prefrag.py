#!/usr/bin/env python3
"""PF vs LDS-built operands: where do the gradient slabs differ (columns, magnitude), and is each path
deterministic run to run?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.ops import _lib  # noqa: E402
from crossscale_ecg.ops.fused_tiny import tiny_step_grads, tiny_forward, labels_int32, new_wprep  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    B, N = 16, 64
    x = torch.randn(N, 500, device=dev)
    y = torch.randint(0, 2, (N,), device=dev)
    idx = torch.randperm(N, device=dev)[:B].int()
    flat = TinyECG().to(dev).flatten_parameters()
    y32 = labels_int32(y, 2)
    a = [tiny_step_grads(flat, x, y32, idx, B, 2, prefrag=True).clone() for _ in range(3)]
    b = [tiny_step_grads(flat, x, y32, idx, B, 2, prefrag=False).clone() for _ in range(3)]
    torch.cuda.synchronize()
    print("PF deterministic:", all(torch.equal(a[0], t) for t in a), " LDS deterministic:",
          all(torch.equal(b[0], t) for t in b))
    d = (a[0] - b[0]).abs()
    cols = (d.amax(0) > 0).nonzero().flatten().tolist()
    rows = (d.amax(1) > 0).nonzero().flatten().tolist()
    print("differing columns:", len(cols), cols[:40], "... rows:", rows)
    print("max abs diff", d.max().item(), "max |ref|", b[0].abs().max().item())
    fa = tiny_forward(flat, x, idx, B, 2, prefrag=True)
    fb = tiny_forward(flat, x, idx, B, 2, prefrag=False)
    print("forward equal:", torch.equal(fa, fb), (fa - fb).abs().max().item())
    # the image itself vs a host-side reference build
    w = new_wprep(dev)
    _lib.check(_lib.kernels().ecg_tiny_prep(flat.data_ptr(), w.data_ptr(), _lib.stream_ptr(dev)), "prep")
    torch.cuda.synchronize()
    img = w[:6400].view(torch.bfloat16).float().cpu()
    p = flat.detach().cpu()
    fragF = img[:1536].view(3, 64, 8)
    bad = 0
    for e in range(1280):
        co, ci, k = e // 80, (e // 5) % 16, e % 5
        rf = 16 * k + ci
        v = fragF[rf >> 5, 16 * ((rf & 31) >> 3) + co, rf & 7].item()
        if v != p[128 + e].to(torch.bfloat16).float().item():
            bad += 1
    print("fragF mismatches vs host build:", bad)
    b2 = w[6400:6464].view(torch.float32).cpu()
    print("b2 equal:", torch.equal(b2, p[1408:1424]))


if __name__ == "__main__":
    main()
