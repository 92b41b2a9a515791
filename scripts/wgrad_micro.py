#!/usr/bin/env python3
"""Weight-gradient kernel on the ResNet1D-34 stride-1 stage shapes (B=1024, k=3, pad 1): mean time of N back-to-back
launches of the split-K kernel, then of its partial reduce (the plan's REDUCE_WGRAD op), TFLOP/s of the kernel.
ECG_WGRAD_TS=0|1 picks the one-tap or the tap-shared kernel (conv1d_mc.hip); splits follow the engine's plan."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import _lib  # noqa: E402
from crossscale_ecg.ops import conv_mc  # noqa: E402

SHAPES = [(1024, 125, 64), (1024, 63, 128), (1024, 32, 256), (1024, 16, 512)]
OP_REDUCE_WGRAD, OP_WORDS = 3, 32


def splits_for(lib, B, L, C):
    s = lib.ecg_conv1d_nlc_wgrad_splits(B, L, C, L, C, 3, 1, 1)
    if s:
        return s, "ts"
    chunks = (B * L + 63) // 64
    tiles = lib.ecg_conv1d_nlc_wgrad_tiles(C, 3, C)
    target = lib.ecg_conv1d_nlc_wgrad_target_wgs(C, 3, C, B, L, L)
    return max(1, min(64, 256, max(1, chunks // 8), max(1, target // tiles))), "one-tap"


def main(reps=50):
    dev = torch.device("cuda:0")
    lib = conv_mc._lib_k()
    _lib._sig(lib, "ecg_plan_run", [_lib.vp, _lib.i32, ctypes.POINTER(ctypes.c_int), _lib.vp])
    torch.manual_seed(0)
    stream = _lib.stream_ptr(dev)
    for B, L, C in SHAPES:
        x = torch.randn(B, L, C, device=dev).bfloat16()
        dy = torch.randn(B, L, C, device=dev).bfloat16()
        S, kind = splits_for(lib, B, L, C)
        part = torch.empty((S, C, 3 * C), dtype=torch.float32, device=dev)
        grad = torch.empty((C, C, 3), dtype=torch.float32, device=dev)
        op = torch.zeros((1, OP_WORDS), dtype=torch.int64)
        op[0, :7] = torch.tensor([OP_REDUCE_WGRAD, part.data_ptr(), S, C, 3, C, grad.data_ptr()])
        bad = ctypes.c_int(-1)

        def wg():
            _lib.check(lib.ecg_conv1d_nlc_wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr(), S, B, L, C, L, C, 3, 1, 1,
                                                stream), "wgrad")

        def red():
            _lib.check(lib.ecg_plan_run(op.data_ptr(), 1, ctypes.byref(bad), stream), "reduce")

        res = []
        for fn in (wg, red):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / reps)
        ref = torch.nn.grad.conv1d_weight(x.float().transpose(1, 2), (C, C, 3), dy.float().transpose(1, 2), 1, 1)
        err = ((grad - ref).norm() / ref.norm()).item()
        flop = 2.0 * B * L * C * 3 * C
        print(f"[{kind}] R={B * L:6d} C={C:3d} S={S:4d}: wgrad {res[0]:7.2f} us ({flop / res[0] / 1e6:6.1f} TF/s) "
              f"reduce {res[1]:6.2f} us  partials {part.numel() * 4 / 1e6:6.1f} MB  rel.err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
