#!/usr/bin/env python3
"""Kernel-level timing of the MFMA NLC conv kernels on the ResNet1D-34 shapes (B=4096, L=500): forward,
data-grad (same kernel, dilated) and weight-grad, back-to-back launches timed with HIP events."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import conv_mc  # noqa: E402

SHAPES = [  # name, B, Lin, Cin, Cout, K, stride, pad
    ("l1", 4096, 125, 64, 64, 3, 1, 1),
    ("l2", 4096, 63, 128, 128, 3, 1, 1),
    ("l3", 4096, 32, 256, 256, 3, 1, 1),
    ("l4", 4096, 16, 512, 512, 3, 1, 1),
    ("l4s", 4096, 32, 256, 512, 3, 2, 1),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3  # us


if __name__ == "__main__":
    for name, B, L, Ci, Co, K, s, p in SHAPES:
        Lo = conv_mc.out_len(L, K, s, p)
        x = torch.randn(B, L, Ci, device="cuda").bfloat16()
        w = torch.randn(Co, K, Ci, device="cuda").bfloat16()
        dy = torch.randn(B, Lo, Co, device="cuda").bfloat16()
        wd = torch.randn(Ci, K, Co, device="cuda").bfloat16()
        fl = 2.0 * B * Lo * Co * Ci * K
        tf = timeit(lambda: conv_mc.fwd_raw(x, w, None, s, p, Lo))
        td = timeit(lambda: conv_mc.fwd_raw(dy, wd, None, 1, K - 1 - p, L, in_dil=s))
        tw = timeit(lambda: conv_mc.wgrad_raw(dy, x, K, s, p))
        print(json.dumps({"shape": name, "fwd_us": round(tf, 1), "fwd_tflops": round(fl / tf / 1e6, 1),
                          "dgrad_us": round(td, 1), "dgrad_tflops": round(fl / td / 1e6, 1),
                          "wgrad_us": round(tw, 1), "wgrad_tflops": round(fl / tw / 1e6, 1)}), flush=True)
