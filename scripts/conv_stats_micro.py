#!/usr/bin/env python3
"""Forward conv1d_nlc on the 64/128-channel ResNet1D-34 stage shapes (B=1024, k=3, stride 1): plain store vs the
BatchNorm-statistics epilogue, one-tile vs multi-tile workgroups (conv_mc.set_multi_tile), mean of N back-to-back
launches (hipEvents).  Separates the cost of the statistics epilogue from the main loop."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import conv_mc  # noqa: E402

SHAPES = [(1024, 125, 64), (1024, 63, 128), (1024, 32, 256)]


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    torch.manual_seed(0)
    for B, L, C in SHAPES:
        x = torch.randn(B, L, C, device="cuda").bfloat16()
        w = (torch.randn(C, 3, C, device="cuda") * 0.05).bfloat16()
        for mode in (0, 1, 2):
            conv_mc.set_multi_tile(mode)
            t_plain = timeit(lambda: conv_mc.fwd_raw(x, w, None, 1, 1, L))
            t_stats = timeit(lambda: conv_mc.fwd_stats_raw(x, w, 1, 1, L))
            rows = conv_mc.stat_rows(B, L, C, L, C)
            print(f"M={B * L:6d} C={C:3d} mt={mode}: plain {t_plain:6.2f} us  stats {t_stats:6.2f} us  "
                  f"({rows} partial rows)", flush=True)
    conv_mc.set_multi_tile(1)


if __name__ == "__main__":
    main()
