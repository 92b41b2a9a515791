#!/usr/bin/env python3
"""ResNet1D-34 B=1024 step time with the weight-gradient ops on a side stream vs one stream, eager plan run vs
graph replay (ECG_RESNET_SIDE is read when the engine is built)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.resnet1d import resnet1d34  # noqa: E402
from crossscale_ecg.ops.resnet_engine import ResNetStepEngine  # noqa: E402


def run(side: str, graph: bool, B=1024, steps=20):
    os.environ["ECG_RESNET_SIDE"] = side
    torch.manual_seed(0)
    m = resnet1d34().cuda()
    eng = ResNetStepEngine(m, B, 500, use_graph=graph)
    eng.set_batch(torch.randn(B, 1, 500, device="cuda"), torch.randint(0, 2, (B,), device="cuda"))
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / steps
    print(f"side={side} graph={graph}: {ms:.3f} ms/step", flush=True)
    del eng, m
    torch.cuda.empty_cache()


if __name__ == "__main__":
    for graph in (False, True):
        for side in ("0", "1"):
            run(side, graph)
