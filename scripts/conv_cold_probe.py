#!/usr/bin/env python3
"""Conv kernel time with the operands in HBM vs resident in the Infinity Cache.

``scripts/r4_conv_probe.py`` replays one conv on the same tensors, so from the second launch on its ~16 MB input is
served by the 256 MB Infinity Cache; inside a ResNet1D-34 step every conv reads an activation written several hundred
MB of traffic earlier (HBM).  This probe times each shape both ways: ``warm`` = the same input / output every launch,
``cold`` = a ring of buffers whose total (input + output) exceeds the Infinity Cache, cycled launch to launch.  Both
are graph-replayed back-to-back launches of the forward conv with the BatchNorm-statistics epilogue, so the host
launch path is out of the picture.  One JSON line per (shape, kernel setting).

    python scripts/conv_cold_probe.py [reps=24]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import conv_mc  # noqa: E402

SHAPES = [("l1", 125, 64, 64), ("l2", 63, 128, 128), ("l3", 32, 256, 256), ("l4", 16, 512, 512)]
B = 1024
RING_MB = 640  # > 256 MB Infinity Cache


def graph_time(fns, reps):
    for f in fns[:3]:
        f()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(reps):
                fns[i % len(fns)]()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (3 * reps) * 1e3


def make_tail(dev, T, C, n, stop=0, gs=None):
    """A device BnTail blob (csrc/include/bn_tail.h) with one forward finalize, packed as the ResNet engine packs it:
    the launch then also runs the fused BatchNorm finalize (the in-step configuration of every statistics conv)."""
    import struct
    gs = gs or max(8, -(-T // 32))
    NG = (T + gs - 1) // gs
    keep = [torch.zeros((C // 64) * (NG + 1), dtype=torch.int32, device=dev),
            torch.zeros((C // 64) * NG * 3 * 64, dtype=torch.float64, device=dev),
            torch.ones(C, device=dev), torch.zeros(C, device=dev)] + [torch.zeros(C, device=dev) for _ in range(6)]
    cnt, gpart, gam, bet, mean, rstd, scale, shift, rm, rv = keep
    P = lambda t: t.data_ptr()  # noqa: E731
    fin = struct.pack("<qqddd12q", 0, 1, float(n), 1e-5, 0.1, P(gam), P(bet), P(mean), P(rstd), P(scale), P(shift),
                      P(rm), P(rv), 0, 0, 0, 0)
    blob = struct.pack("<qqqq", P(cnt), P(gpart), gs, 1 | (stop << 8)) + fin
    blob += b"\0" * (304 - len(blob))
    dt = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev)
    keep.append(dt)
    return dt.data_ptr(), keep


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for name, L, Ci, Co in SHAPES:
        mb = B * L * (Ci + Co) * 2 / 2 ** 20
        nbuf = max(2, int(RING_MB / mb) + 1)
        xs = [torch.randn(B, L, Ci, device=dev).bfloat16() for _ in range(nbuf)]
        w = (torch.randn(Co, 3, Ci, device=dev) * 0.05).bfloat16()
        settings = [("tap64", 1), ("multi_tile", 0)] if Ci == Co == 64 else [("tap", None)]
        for label, t64 in settings:
            if t64 is not None:
                conv_mc.set_tap64(bool(t64))
            rows = conv_mc.stat_rows(B, L, Ci, L, Co)
            ys = [torch.empty(B, L, Co, device=dev, dtype=torch.bfloat16) for _ in range(nbuf)]
            st = torch.empty(2, rows, Co, device=dev)
            lib = conv_mc._lib_k()

            def mk(i):
                def f():
                    lib.ecg_conv1d_nlc_fwd_ex(xs[i].data_ptr(), w.data_ptr(), None, ys[i].data_ptr(), st.data_ptr(),
                                              None, None, B, L, Ci, L, Co, 3, 1, 1, 1, 0, None, None,
                                              torch.cuda.current_stream().cuda_stream)
                return f
            fns = [mk(i) for i in range(nbuf)]
            warm = graph_time(fns[:1], reps)
            cold = graph_time(fns, max(reps, nbuf))
            tails = {}
            # full tail; diagnostic exits after the level-1 / level-2 tickets (bn_tail.h); one level-1 group
            for key, kw in (("warm_tail_us", {}), ("tail_stop1_us", {"stop": 1}), ("tail_stop2_us", {"stop": 2}),
                            ("tail_stop3_us", {"stop": 3}),
                            ("tail_1group_us", {"gs": rows})):
                tail_ptr, keep = make_tail(dev, rows, Co, B * L, **kw)

                def ft():
                    lib.ecg_conv1d_nlc_fwd_ex(xs[0].data_ptr(), w.data_ptr(), None, ys[0].data_ptr(), st.data_ptr(),
                                              None, None, B, L, Ci, L, Co, 3, 1, 1, 1, 0, None, tail_ptr,
                                              torch.cuda.current_stream().cuda_stream)
                tails[key] = round(graph_time([ft], reps), 2)
                del keep
            print(json.dumps({"shape": name, "kernel": label, "B": B, "io_mb": round(mb, 1), "ring": nbuf,
                              "stat_rows": rows, "warm_us": round(warm, 2), **tails, "cold_us": round(cold, 2),
                              "cold_tbs": round(mb * 2 ** 20 / (cold * 1e-6) / 1e12, 2)}), flush=True)
        conv_mc.set_tap64(True)
        del xs


if __name__ == "__main__":
    main()
