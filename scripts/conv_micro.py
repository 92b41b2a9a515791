#!/usr/bin/env python3
"""Forward conv1d_nlc on the four ResNet1D-34 stage shapes (B=1024, k=3, stride 1, pad 1): mean time of N
back-to-back launches, TFLOP/s and compulsory-byte TB/s.  The tile family follows ECG_CONV_TILE / the picker."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops.conv_mc import fwd_raw  # noqa: E402

SHAPES = [(1024, 125, 64), (1024, 63, 128), (1024, 32, 256), (1024, 16, 512)]


def main(reps=50):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    tag = os.environ.get("ECG_CONV_TILE", "picker") + "|v128=" + os.environ.get("ECG_CONV_V128", "0")
    for B, L, C in SHAPES:
        x = torch.randn(B, L, C, device=dev).bfloat16()
        w = (torch.randn(C, 3, C, device=dev) * 0.05).bfloat16()
        fwd_raw(x, w, None, 1, 1, L)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fwd_raw(x, w, None, 1, 1, L)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        flop = 2.0 * B * L * C * 3 * C
        nb = 2.0 * (2 * B * L * C + 3 * C * C)
        print(f"[{tag}] M={B * L:6d} C={C:3d}: {us:7.2f} us  {flop / us / 1e6:6.1f} TFLOP/s  {nb / us / 1e6:5.2f} TB/s",
              flush=True)


if __name__ == "__main__":
    main()
