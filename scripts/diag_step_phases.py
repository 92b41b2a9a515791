#!/usr/bin/env python3
"""Diagnostic: where the fused TinyECG step spends its cycles (s_memtime stamps, wave 0 of each WG).

Phases: 0 stage x/params | 1 conv1 | 2 conv2 fwd + mask | 3 head || mask-weighted wgrad | 4 dgrad2 + wgrad1 |
5 row store.  Reports
  * hipEvent times of the gradient-only kernel and the two-launch round (LDS-built and prepared operands);
  * the per-step kernel's phases cold (first pass of a launch) and warm (MODE 2: the same workgroup computes
    its sample again right after, with warm instruction / scalar / data caches);
Stamped runs are slower than real ones: read shares, not totals.
"""
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


def phase_table(s, k0, names, label):
    print(label)
    for k, name in enumerate(names):
        d = (s[:, k0 + k + 1] - s[:, k0 + k]).double().tolist()
        print(f"  phase {k} {name:>14s}: median {statistics.median(d):8.0f} cyc  max {max(d):8.0f}")
    tot = (s[:, k0 + len(names)] - s[:, k0]).double().tolist()
    print(f"  total            : median {statistics.median(tot):8.0f} cyc")


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
    for pf in (False, True):
        t = ev_time(lambda: tiny_step_grads(flat, x, y32, idx, B, 2, slab, prefrag=pf), 200)
        print(f"gradient-only kernel (eager loop, prefrag={pf}, PF adds the prep launch): {t:.2f} us")
    for name, kw in (("two-launch LDS", dict(prefrag=False)), ("two-launch PF ", dict(prefrag=True))):
        m = TinyECG().to(dev)
        tr = FusedTinyTrainer(m, x, y, B, 50, seed=0, **kw)
        tr.run_round()
        torch.cuda.synchronize()
        t = ev_time(lambda: tr.run_round(), 20) / 50
        tr.use_graph = False
        te = ev_time(lambda: tr.run_round(), 4) / 50
        print(f"{name} round: graph {t:.2f} us/step, eager {te:.2f} us/step")
        tr.close()

    # the production kernel (MODE 0, 16 waves at L=500) stamped in a single, cold pass
    for label, pf in (("LDS-built operands", False), ("prepared fragments (PF)", True)):
        st = torch.zeros(B * 16, dtype=torch.int64, device=dev)
        wp = torch.zeros(lib.ecg_tiny_wprep_bytes(), dtype=torch.uint8, device=dev)
        for _ in range(5):
            st.zero_()
            lib.ecg_tiny_set_stamps(st.data_ptr())
            tiny_step_grads(flat, x, y32, idx, B, 2, slab, prefrag=pf, wprep=wp if pf else None)
            torch.cuda.synchronize()
            lib.ecg_tiny_set_stamps(None)
        phase_table(st.view(B, 16).cpu(), 0, NAMES, f"[{label}] PRODUCTION per-step kernel (16 waves), cold:")

    # cold vs warm passes of the per-step kernel (MODE 2, 8 waves), operands built in LDS vs prepared fragments
    wprep = torch.empty(lib.ecg_tiny_wprep_bytes(), dtype=torch.uint8, device=dev)
    for label, wp in (("LDS-built operands", None), ("prepared fragments (PF)", wprep.data_ptr())):
        st = torch.zeros(B * 16, dtype=torch.int64, device=dev)
        lib.ecg_tiny_set_stamps(st.data_ptr())
        for _ in range(5):
            st.zero_()
            _lib.check(lib.ecg_tiny_step_grads_twice(x.data_ptr(), L, x.stride(0), idx.data_ptr(), y32.data_ptr(),
                                                     flat.data_ptr(), 2, slab.data_ptr(), slab.shape[1], B, 1.0 / B,
                                                     0, wp, _lib.stream_ptr(dev)), "twice")
        torch.cuda.synchronize()
        lib.ecg_tiny_set_stamps(None)
        s = st.view(B, 16).cpu()
        cyc = (s[:, 6] - s[:, 0]).double()
        rt = (s[:, 14] - s[:, 15]).double() * 10.0  # 100 MHz -> ns (both passes)
        ghz = statistics.median(((s[:, 13] - s[:, 0]).double() / rt).tolist())
        print(f"[{label}] in-kernel clock ~{ghz:.2f} GHz")
        phase_table(s, 0, NAMES, f"[{label}] per-step kernel, COLD pass (fresh launch):")
        phase_table(s, 7, NAMES, f"[{label}] per-step kernel, WARM pass (same workgroup, immediately after):")
        print(f"  cold total median {statistics.median(cyc.tolist()):.0f} cyc")


if __name__ == "__main__":
    main()
