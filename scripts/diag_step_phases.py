#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the fused TinyECG step (s_memtime stamps, wave 0 of each WG).

Phases: 0 stage x/params | 1 conv1 | 2 conv2 fwd + mask | 3 head || mask-weighted wgrad | 4 dgrad2 + wgrad1 |
5 row store | 6 (final reducer only) reduction tree + SGD.  Also hipEvent times of the single-launch step,
the gradient-only kernel, the two-launch path and graph rounds.  Stamped runs are slower than real ones:
read shares, not totals.
"""
import ctypes as C
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crossscale_ecg  # noqa: E402
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.ops import _lib  # noqa: E402
from crossscale_ecg.ops.fused_tiny import tiny_step_grads, labels_int32, slab_stride, FusedTinyTrainer  # noqa: E402

NAMES = ["stage", "conv1", "conv2+mask", "head||M", "dgrad2+wgrad1", "row store"]


def ev_time(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    dev = torch.device("cuda:0")
    B, L, N = 256, int(os.environ.get("DIAG_L", 500)), 20000
    x = torch.randn(N, L, device=dev)
    y = torch.zeros(N, dtype=torch.long, device=dev)
    model = TinyECG().to(dev)
    flat = model.flatten_parameters()
    y32 = labels_int32(y, 2)
    idx = torch.randperm(N, device=dev)[:B].int()
    lib = _lib.kernels()
    slab = torch.empty(B, slab_stride(2), device=dev)
    print(f"gradient-only kernel (eager loop): {ev_time(lambda: tiny_step_grads(flat, x, y32, idx, B, 2, slab), 200):.2f} us")
    for single in (True, False):
        m = TinyECG().to(dev)
        tr = FusedTinyTrainer(m, x, y, B, 50, seed=0, single_launch=single)
        tr.run_round()
        torch.cuda.synchronize()
        t = ev_time(lambda: tr.run_round(), 10) / 50
        tr.use_graph = False
        te = ev_time(lambda: tr.run_round(), 4) / 50
        print(f"{'single-launch' if single else 'two-launch  '} step: graph {t:.2f} us/step, eager {te:.2f} us/step")
        tr.close()
    # stamped run of the single-launch step
    m = TinyECG().to(dev)
    tr = FusedTinyTrainer(m, x, y, B, 1, seed=0, use_graph=False)
    st = torch.zeros(B * 16, dtype=torch.int64, device=dev)
    lib.ecg_tiny_set_stamps(st.data_ptr())
    for _ in range(5):
        st.zero_()
        tr.run_round()
    torch.cuda.synchronize()
    lib.ecg_tiny_set_stamps(None)
    tr.close()
    s = st.view(B, 16).cpu()
    cyc = (s[:, 6] - s[:, 0]).double()
    rt = (s[:, 14] - s[:, 15]).double() * 10.0  # 100 MHz -> ns
    ghz = statistics.median((cyc / rt).tolist())
    print(f"in-kernel clock ~{ghz:.2f} GHz; WG lifetime to row store median {statistics.median(rt.tolist()) / 1e3:.2f} us "
          f"({statistics.median(cyc.tolist()):.0f} cycles)")
    for k in range(6):
        d = (s[:, k + 1] - s[:, k]).double().tolist()
        print(f"  phase {k} {NAMES[k]:>14s}: median {statistics.median(d):8.0f} cyc  max {max(d):8.0f}")
    fin = (s[:, 7] != 0).nonzero().flatten().tolist()
    t0 = s[:, 15].min()
    if fin:
        f = fin[0]
        print(f"  final reducer WG {f}: tree+SGD {int(s[f, 7] - s[f, 6])} cyc; kernel span to final end "
              f"{(s[f, 13] - t0).item() * 10 / 1e3:.2f} us")
    print(f"  WG start spread {(s[:, 15].max() - t0).item() * 10 / 1e3:.2f} us, last row store "
          f"{(s[:, 14].max() - t0).item() * 10 / 1e3:.2f} us")


if __name__ == "__main__":
    main()
