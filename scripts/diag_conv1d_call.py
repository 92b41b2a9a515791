#!/usr/bin/env python3
"""Decompose the Module-2 single-call time (reference ``time_once``: 3 warm-up calls + ONE timed call) of the HIP
conv1d and of torch.nn.Conv1d at B=256, K=7, L=500: Python wrapper, ctypes, launch, kernel, synchronise."""
from __future__ import annotations

import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import _lib  # noqa: E402
from crossscale_ecg.ops.conv1d import conv1d_valid  # noqa: E402


def once(fn, sync=True, reps=41):
    out = []
    for _ in range(reps):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(out)


def main():
    dev = torch.device("cuda:0")
    B, L, K = 256, 500, 7
    x = torch.randn(B, 1, L, device=dev)
    w = torch.randn(K, device=dev)
    out = torch.empty(B, L - K + 1, device=dev)
    conv = torch.nn.Conv1d(1, 1, K, bias=False).to(dev)
    lib = _lib.kernels()
    raw = torch._C._cuda_getCurrentRawStream
    xp, wp, op = x.data_ptr(), w.data_ptr(), out.data_ptr()
    fn = lib.conv1d_batch_hip
    rows = []
    with torch.no_grad():
        rows.append(("torch.cuda.synchronize alone", once(lambda: None)))
        rows.append(("nn.Conv1d + sync", once(lambda: conv(x))))
        rows.append(("nn.Conv1d, no sync (host return)", once(lambda: conv(x), sync=False)))
        rows.append(("conv1d_valid(hip) + sync", once(lambda: conv1d_valid(x[:, 0], w, backend="hip", out=out))))
        rows.append(("conv1d_valid(hip), no sync", once(lambda: conv1d_valid(x[:, 0], w, backend="hip", out=out),
                                                        sync=False)))
        rows.append(("raw ctypes launch + sync", once(lambda: fn(xp, wp, op, B, L, K, raw(0)))))
        rows.append(("raw ctypes launch, no sync", once(lambda: fn(xp, wp, op, B, L, K, raw(0)), sync=False)))
        from crossscale_ecg.ops.conv1d import HipConv1dValid
        bop = HipConv1dValid(w, blocking=True)
        x2 = x[:, 0].contiguous()
        rows.append(("HipConv1dValid (bound, spin) + sync", once(lambda: bop(x2, out))))
        rows.append(("HipConv1dValid (bound, spin), no sync", once(lambda: bop(x2, out), sync=False)))
        rows.append(("spin C call, no sync", once(lambda: lib.conv1d_batch_hip_spin(xp, wp, op, B, L, K, raw(0)),
                                                  sync=False)))
        if hasattr(lib, "conv1d_batch_hip_sync"):
            rows.append(("blocking C call (launch+hipStreamSynchronize)",
                         once(lambda: lib.conv1d_batch_hip_sync(xp, wp, op, B, L, K, raw(0)), sync=False)))
        rows.append(("flag C call (launch + host-mapped completion word)",
                     once(lambda: lib.conv1d_batch_hip_flag(xp, wp, op, B, L, K, raw(0)), sync=False)))
        rows.append(("flag C call + sync", once(lambda: lib.conv1d_batch_hip_flag(xp, wp, op, B, L, K, raw(0)))))
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ks = []
        for _ in range(21):
            ev0.record()
            fn(xp, wp, op, B, L, K, raw(0))
            ev1.record()
            ev1.synchronize()
            ks.append(ev0.elapsed_time(ev1) * 1e3)
        rows.append(("hip kernel, event-timed", statistics.median(ks)))
        ks = []
        for _ in range(21):
            ev0.record()
            conv(x)
            ev1.record()
            ev1.synchronize()
            ks.append(ev0.elapsed_time(ev1) * 1e3)
        rows.append(("nn.Conv1d, event-timed", statistics.median(ks)))
    for name, us in rows:
        print(f"{name:50s} {us:8.2f} us")


if __name__ == "__main__":
    main()
