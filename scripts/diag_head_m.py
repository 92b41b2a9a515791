#!/usr/bin/env python3
"""Diagnostic: in the production TinyECG step kernel's phase 3, when does the head (wave 0) finish vs the
mask-weighted conv2 wgrad waves (1 and the last)?  s_memtime cycles after the phase-3 start stamp."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.ops import _lib  # noqa: E402
from crossscale_ecg.ops.fused_tiny import tiny_step_grads, labels_int32, slab_stride  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, L, N = 256, 500, 20000
    x = torch.randn(N, L, device=dev)
    y = torch.zeros(N, dtype=torch.long, device=dev)
    flat = TinyECG().to(dev).flatten_parameters()
    y32 = labels_int32(y, 2)
    idx = torch.randperm(N, device=dev)[:B].int()
    lib = _lib.kernels()
    slab = torch.empty(B, slab_stride(2), device=dev)
    wp = torch.zeros(lib.ecg_tiny_wprep_bytes(), dtype=torch.uint8, device=dev)
    st = torch.zeros(B * 16, dtype=torch.int64, device=dev)
    for _ in range(5):
        st.zero_()
        lib.ecg_tiny_set_stamps(st.data_ptr())
        tiny_step_grads(flat, x, y32, idx, B, 2, slab, prefrag=True, wprep=wp)
        torch.cuda.synchronize()
        lib.ecg_tiny_set_stamps(None)
    s = st.view(B, 16).cpu().double()
    for name, k in (("head end (wave 0)", 8), ("M end (wave 1)", 9), ("M end (last wave)", 10),
                    ("phase 3 barrier passed", 4)):
        d = (s[:, k] - s[:, 3]).tolist()
        print(f"{name:24s}: median {statistics.median(d):7.0f} cyc  max {max(d):7.0f}")
    for k in range(6):
        d = (s[:, k + 1] - s[:, k]).tolist()
        print(f"phase {k}: median {statistics.median(d):7.0f}")


if __name__ == "__main__":
    main()
