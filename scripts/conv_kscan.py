#!/usr/bin/env python3
"""Fixed vs per-K-step cost of the forward conv: time conv1d_nlc (plain and with the BatchNorm-statistics epilogue)
at a fixed output shape (B, L, Cout) while C_in - hence the number of 64-deep K steps, 3 * C_in / 64 - varies, next
to hipBLASLt (torch.mm) on the same GEMM (M = B*L, K = 3*C_in, N = Cout; the im2col is not timed) as a known-good
reference.  A linear fit of time vs K steps splits the launch into fixed (prologue / epilogue / tail) and streaming
cost.   python scripts/conv_kscan.py [B L Cout]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import conv_mc  # noqa: E402


def _time(fn, reps=40):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = None
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        best = us if best is None else min(best, us)
    return best


def main():
    B, L, Cout = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (1024, 32, 256)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    pts = []
    print(f"B={B} L={L} Cout={Cout}  (us; TF/s)", flush=True)
    for Cin in (64, 128, 256, 512, 1024):
        x = torch.randn(B, L, Cin, device=dev).bfloat16()
        w = (torch.randn(Cout, 3, Cin, device=dev) * 0.05).bfloat16()
        a = torch.randn(B * L, 3 * Cin, device=dev).bfloat16()
        bt = (torch.randn(3 * Cin, Cout, device=dev) * 0.05).bfloat16()
        flop = 2.0 * B * L * Cout * 3 * Cin
        t_plain = _time(lambda: conv_mc.fwd_raw(x, w, None, 1, 1, L))
        t_stats = _time(lambda: conv_mc.fwd_stats_raw(x, w, 1, 1, L))
        t_mm = _time(lambda: torch.mm(a, bt))
        ks = 3 * Cin // 64
        pts.append((ks, t_plain, t_stats, t_mm))
        print(f"Cin={Cin:5d} ksteps={ks:3d}  conv {t_plain:7.2f} ({flop / t_plain / 1e6:6.1f})  conv+stats "
              f"{t_stats:7.2f} ({flop / t_stats / 1e6:6.1f})  torch.mm {t_mm:7.2f} ({flop / t_mm / 1e6:6.1f})",
              flush=True)
    for j, name in ((1, "conv"), (2, "conv+stats"), (3, "torch.mm")):
        n = len(pts)
        sx = sum(p[0] for p in pts)
        sy = sum(p[j] for p in pts)
        sxx = sum(p[0] ** 2 for p in pts)
        sxy = sum(p[0] * p[j] for p in pts)
        slope = (n * sxy - sx * sy) / (n * sxx - sx * sx)
        icpt = (sy - slope * sx) / n
        print(f"fit {name:10s}: {icpt:6.2f} us fixed + {slope:5.3f} us per 64-deep K step", flush=True)


if __name__ == "__main__":
    main()
