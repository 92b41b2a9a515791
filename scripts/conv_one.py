#!/usr/bin/env python3
"""Run one conv shape a few times (for rocprofv3 --pmc counter collection): l1..l4 of conv_microbench."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import conv_mc  # noqa: E402

SH = {"l1": (4096, 125, 64, 64), "l2": (4096, 63, 128, 128), "l3": (4096, 32, 256, 256), "l4": (4096, 16, 512, 512)}
if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "l3"
    B, L, Ci, Co = SH[name]
    x = torch.randn(B, L, Ci, device="cuda").bfloat16()
    w = torch.randn(Co, 3, Ci, device="cuda").bfloat16()
    for _ in range(5):
        conv_mc.fwd_raw(x, w, None, 1, 1, L)
    torch.cuda.synchronize()
    print("ok", name)
