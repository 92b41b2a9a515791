#!/usr/bin/env python3
"""Diagnostic: per-phase cycle breakdown of the fused TinyECG step (s_memtime stamps, wave 0 of each WG).

Phases: 0 stage x/params | 1 conv1 | 2 conv2 fwd + pool | 3 head | 4 dh2 + wgrad2 | 5 dgrad2 + wgrad1 | 6 slab
store.  Prints median cycles per phase over workgroups, the in-kernel clock (s_memtime vs s_memrealtime)
and hipEvent times of both kernels.  Stamped runs are slower than real ones: read shares, not totals.
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

NAMES = ["stage", "conv1", "conv2+pool", "head", "dh2+wgrad2", "dgrad2+wgrad1", "store"]


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
    # plain timing first (no stamps)
    slab = torch.empty(B, slab_stride(2), device=dev)
    for _ in range(20):
        tiny_step_grads(flat, x, y32, idx, B, 2, slab)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        tiny_step_grads(flat, x, y32, idx, B, 2, slab)
    e1.record()
    torch.cuda.synchronize()
    print(f"step kernel (eager loop): {e0.elapsed_time(e1) / 200 * 1e3:.2f} us/launch")
    pc, mom, la = flat.clone(), torch.zeros_like(flat), torch.zeros(1, device=dev)
    strm = _lib.stream_ptr(dev)

    def red():
        lib.ecg_slab_reduce_sgd(slab.data_ptr(), B, slab.shape[1], 1458, pc.data_ptr(), mom.data_ptr(), None,
                                la.data_ptr(), 1e-2, 0.9, 0.0, 0, 1, strm)
    for _ in range(20):
        red()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(200):
        red()
    e1.record()
    torch.cuda.synchronize()
    print(f"reduce+SGD kernel (eager loop, L2-warm slab): {e0.elapsed_time(e1) / 200 * 1e3:.2f} us/launch")
    tr = FusedTinyTrainer(model, x, y, B, 50, seed=0)
    tr.run_round()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        tr.run_round()
    e1.record()
    torch.cuda.synchronize()
    print(f"graph round: {e0.elapsed_time(e1) / 500 * 1e3:.2f} us/step (step kernel + reduce/SGD)")
    tr.close()
    # stamped run
    st = torch.zeros(B * 16, dtype=torch.int64, device=dev)
    lib.ecg_tiny_set_stamps.argtypes = [C.c_void_p]
    lib.ecg_tiny_set_stamps(st.data_ptr())
    for _ in range(5):
        tiny_step_grads(flat, x, y32, idx, B, 2, slab)
    torch.cuda.synchronize()
    lib.ecg_tiny_set_stamps(None)
    s = st.view(B, 16).cpu()
    cyc = (s[:, 7] - s[:, 0]).double()
    rt = (s[:, 14] - s[:, 15]).double() * 10.0  # 100 MHz -> ns
    ghz = statistics.median((cyc / rt).tolist())
    print(f"in-kernel clock ~{ghz:.2f} GHz; WG lifetime median {statistics.median(rt.tolist()) / 1e3:.2f} us "
          f"({statistics.median(cyc.tolist()):.0f} cycles)")
    for k in range(7):
        d = (s[:, k + 1] - s[:, k]).double().tolist()
        print(f"  phase {k} {NAMES[k]:>14s}: median {statistics.median(d):8.0f} cyc  max {max(d):8.0f}")
    starts = (s[:, 15] - s[:, 15].min()).double() * 10.0
    ends = (s[:, 14] - s[:, 15].min()).double() * 10.0
    print(f"  WG start spread {starts.max().item() / 1e3:.2f} us, last end {ends.max().item() / 1e3:.2f} us")


if __name__ == "__main__":
    main()
