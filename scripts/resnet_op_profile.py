#!/usr/bin/env python3
"""Per-op timing of the native ResNet1D step plan (hipEvents around N back-to-back launches of ONE plan op, after
the whole step ran once): time, FLOP rate and activation bytes per conv / wgrad / BN op, sorted by total time.
Usage: resnet_op_profile.py [depth=34] [B=1024]"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.resnet1d import resnet1d18, resnet1d34  # noqa: E402
from crossscale_ecg.ops.resnet_engine import OP, ResNetStepEngine  # noqa: E402

KIND = {v: k for k, v in OP.items()}


def main(depth=34, B=1024, reps=20):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = (resnet1d34 if depth == 34 else resnet1d18)().to(dev)
    eng = ResNetStepEngine(m, B, 500, use_graph=False)
    eng.set_batch(torch.randn(B, 1, 500, device=dev), torch.randint(0, 2, (B,), device=dev))
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    ops = eng.ops.tolist()
    rows = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i, o in enumerate(ops):
        kind = KIND[o[0]]
        eng._run(i, i + 1)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            eng._run(i, i + 1)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        flop, desc, nbytes = 0.0, "", 0.0
        if kind == "CONV_FWD":
            Bq, Lin, Cin, Lout, Cout, K, s, p, dil = o[8:17]
            M = Bq * Lout
            flop = 2.0 * M * Cout * K * Cin / (dil if dil > 1 else 1)
            nbytes = 2.0 * (Bq * Lin * Cin + M * Cout + Cout * K * Cin)
            desc = f"{'dgrad' if o[19] or dil > 1 or o[6] else 'fwd'} M={M} N={Cout} K={K}x{Cin} s={s} dil={dil}"
        elif kind == "CONV_WGRAD":
            S, Bq, Lin, Cin, Lout, Cout, K = o[4:11]
            flop = 2.0 * Bq * Lout * Cout * K * Cin
            nbytes = 2.0 * (Bq * Lin * Cin + Bq * Lout * Cout) + 4.0 * S * Cout * K * Cin
            desc = f"wgrad R={Bq * Lout} Cout={Cout} K={K}x{Cin} splits={S}"
        elif kind == "REDUCE_WGRAD":
            desc = f"S={o[2]} |dW|={o[3] * o[4] * o[5]}"
        rows.append((us, kind, desc, flop, nbytes))
    tot = sum(r[0] for r in rows)
    print(f"ResNet1D-{depth} B={B}: {len(rows)} ops, sum of per-op times {tot / 1e3:.3f} ms "
          f"(back-to-back single-op launches; the captured step graph overlaps nothing, so this is an upper bound)")
    by = collections.defaultdict(lambda: [0.0, 0])
    for us, kind, desc, flop, _ in rows:
        by[kind][0] += us
        by[kind][1] += 1
    for k, (us, n) in sorted(by.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k:16s} {n:4d} ops {us / 1e3:7.3f} ms ({100 * us / tot:5.1f} %)")
    print("slowest conv / wgrad ops:")
    for us, kind, desc, flop, nb in sorted([r for r in rows if r[3] > 0], key=lambda r: -r[0])[:25]:
        print(f"  {us:8.1f} us  {flop / us / 1e6:7.1f} TFLOP/s  {nb / us / 1e6:6.2f} TB/s  {kind:10s} {desc}")
    print("all ops grouped by shape (count, total, mean, TFLOP/s, TB/s of the compulsory bytes):")
    grp = collections.OrderedDict()
    for us, kind, desc, flop, nb in rows:
        g = grp.setdefault((kind, desc), [0, 0.0, flop, nb])
        g[0] += 1
        g[1] += us
    for (kind, desc), (n, us, flop, nb) in sorted(grp.items(), key=lambda kv: -kv[1][1]):
        mean = us / n
        rate = f"{flop / mean / 1e6:7.1f} TF/s" if flop else " " * 12
        bw = f"{nb / mean / 1e6:6.2f} TB/s" if nb else " " * 11
        print(f"  {n:3d} x {mean:7.1f} us = {us:7.1f} us  {rate} {bw}  {kind:14s} {desc}")


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:]]
    main(*a)
