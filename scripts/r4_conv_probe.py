#!/usr/bin/env python3
"""Kernel-level timing of the ResNet1D-34 conv shapes at the bench batch (B=1024) and at B=4096: forward (no
statistics), forward with the BatchNorm-statistics epilogue, data-grad (unstrided and strided) and the weight-gradient
split-K kernel (partials only, the engine's split plan), each as the mean GPU time of back-to-back launches
replayed from a captured graph.  Prints one JSON line per (shape, batch).

    python scripts/r4_conv_probe.py [reps=30] [batches=1024,4096]
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import _lib, conv_mc  # noqa: E402

# name, Lin, Cin, Cout, K, stride, pad   (ResNet1D-34 at L=500: stem -> 250 -> pool -> 125)
SHAPES = [("l1", 125, 64, 64, 3, 1, 1), ("l2", 63, 128, 128, 3, 1, 1), ("l3", 32, 256, 256, 3, 1, 1),
          ("l4", 16, 512, 512, 3, 1, 1), ("l2s", 125, 64, 128, 3, 2, 1), ("l3s", 63, 128, 256, 3, 2, 1),
          ("l4s", 32, 256, 512, 3, 2, 1)]


def timeit(fn, reps):
    """Mean GPU time per call: ``reps`` calls captured into one hipGraph and replayed, so the host-side launch cost
    of the Python/ctypes path (~10 us, more than the smaller kernels) does not starve the GPU between kernels."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * reps) * 1e3  # us


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    batches = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "1024,4096").split(",")]
    lib = conv_mc._lib_k()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for B in batches:
        for name, L, Ci, Co, K, s, p in SHAPES:
            Lo = conv_mc.out_len(L, K, s, p)
            x = torch.randn(B, L, Ci, device=dev).bfloat16()
            w = (torch.randn(Co, K, Ci, device=dev) * 0.05).bfloat16()
            dy = torch.randn(B, Lo, Co, device=dev).bfloat16()
            wd = (torch.randn(Ci, K, Co, device=dev) * 0.05).bfloat16()
            fl = 2.0 * B * Lo * Co * Ci * K
            rec = {"shape": name, "B": B, "M": B * Lo, "Cin": Ci, "Cout": Co, "stride": s, "gflop": round(fl / 1e9, 2)}
            rec["fwd_us"] = timeit(lambda: conv_mc.fwd_raw(x, w, None, s, p, Lo), reps)
            rec["fwd_stats_us"] = timeit(lambda: conv_mc.fwd_stats_raw(x, w, s, p, Lo), reps)
            rec["dgrad_us"] = timeit(lambda: conv_mc.fwd_raw(dy, wd, None, 1, K - 1 - p, L, in_dil=s), reps)
            R = B * Lo
            chunks = (R + 63) // 64
            tiles = lib.ecg_conv1d_nlc_wgrad_tiles(Co, K, Ci)
            splits = lib.ecg_conv1d_nlc_wgrad_splits(B, L, Ci, Lo, Co, K, s, p)
            if not splits:
                target = lib.ecg_conv1d_nlc_wgrad_target_wgs(Co, K, Ci, B, L, Lo)
                splits = max(1, min(256, max(1, chunks // 8), max(1, target // max(1, tiles))))
            part = torch.empty((splits, Co, K * Ci), dtype=torch.float32, device=dev)
            def wg():
                _lib.check(lib.ecg_conv1d_nlc_wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr(), splits, B, L, Ci, Lo,
                                                    Co, K, s, p, _lib.stream_ptr(dev)), "wgrad")
            rec["wgrad_us"] = timeit(wg, reps)
            rec["wgrad_splits"] = splits
            rec["wgrad_part_mb"] = round(part.numel() * 4 / 2**20, 1)
            for k in ("fwd", "fwd_stats", "dgrad", "wgrad"):
                rec[k + "_us"] = round(rec[k + "_us"], 2)
                rec[k + "_tf"] = round(fl / rec[k + "_us"] / 1e6, 1)
            print(json.dumps(rec), flush=True)
            del x, w, dy, wd, part


if __name__ == "__main__":
    main()
