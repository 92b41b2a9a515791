"""ResNet1D stress benchmark (BASELINE.json config 5): per-layer conv timings (MFMA NLC kernels vs MIOpen)
and full training-step throughput of ResNet1D-34 with the ``hip`` and ``torch`` backends, bf16."""
from __future__ import annotations

import time
from typing import Dict, List

import torch
import torch.nn.functional as F

from ..models.resnet1d import resnet1d34
from ..ops.conv_mc import conv1d_nlc, out_len

# (name, B, L_in, C_in, C_out, K, stride, pad) at batch 256, L=500 -> after stem L=125
LAYERS = [
    ("layer1.conv", 256, 125, 64, 64, 3, 1, 1),
    ("layer2.0.conv1", 256, 125, 64, 128, 3, 2, 1),
    ("layer2.conv", 256, 63, 128, 128, 3, 1, 1),
    ("layer3.0.conv1", 256, 63, 128, 256, 3, 2, 1),
    ("layer3.conv", 256, 32, 256, 256, 3, 1, 1),
    ("layer4.0.conv1", 256, 32, 256, 512, 3, 2, 1),
    ("layer4.conv", 256, 16, 512, 512, 3, 1, 1),
    ("layer4.0.down", 256, 32, 256, 512, 1, 2, 0),
]


def _ev(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


def layer_table(dev="cuda") -> List[Dict]:
    rows = []
    for name, B, L, Cin, Cout, K, s, p in LAYERS:
        x = torch.randn(B, L, Cin, device=dev).bfloat16().requires_grad_(True)
        w = torch.randn(Cout, Cin, K, device=dev, requires_grad=True)
        xc = x.detach().transpose(1, 2).contiguous().requires_grad_(True)
        wb = w.detach().bfloat16().requires_grad_(True)
        Lo = out_len(L, K, s, p)
        flops = 2 * B * Lo * Cout * Cin * K
        hf = _ev(lambda: conv1d_nlc(x, w, None, s, p))
        tf = _ev(lambda: F.conv1d(xc, wb, None, s, p))
        y = conv1d_nlc(x, w, None, s, p)
        g = torch.randn_like(y)
        yt = F.conv1d(xc, wb, None, s, p)
        gt = torch.randn_like(yt)
        hb = _ev(lambda: torch.autograd.grad(conv1d_nlc(x, w, None, s, p), (x, w), g))
        tb = _ev(lambda: torch.autograd.grad(F.conv1d(xc, wb, None, s, p), (xc, wb), gt))
        rows.append({"layer": name, "B": B, "L": L, "Cin": Cin, "Cout": Cout, "K": K, "stride": s,
                     "hip_fwd_ms": hf, "miopen_fwd_ms": tf, "hip_fwd_tflops": flops / hf / 1e9,
                     "miopen_fwd_tflops": flops / tf / 1e9, "hip_fwdbwd_ms": hb, "miopen_fwdbwd_ms": tb,
                     "speedup_fwd": tf / hf, "speedup_fwdbwd": tb / hb})
    return rows


def train_throughput(backend: str, B: int = 256, L: int = 500, steps: int = 20, dev="cuda") -> float:
    torch.manual_seed(0)
    m = resnet1d34(backend=backend).to(dev)
    opt = torch.optim.SGD(m.parameters(), lr=1e-2, momentum=0.9)
    x = torch.randn(B, 1, L, device=dev)
    y = torch.randint(0, 2, (B,), device=dev)

    def step():
        opt.zero_grad(set_to_none=True)
        if backend == "torch":
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = F.cross_entropy(m(x), y)
        else:
            loss = F.cross_entropy(m(x), y)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return B * steps / (time.perf_counter() - t0)


def engine_throughput(B: int = 256, L: int = 500, steps: int = 20, warmup: int = 3, depth: int = 34,
                      use_graph: bool = True, dev="cuda") -> float:
    """Samples/s of the native step engine (ops.resnet_engine): fwd + bwd + SGD per step, bf16, one hipGraph."""
    from ..models.resnet1d import resnet1d18
    from ..ops.resnet_engine import ResNetStepEngine
    torch.manual_seed(0)
    m = (resnet1d34 if depth == 34 else resnet1d18)().to(dev)
    eng = ResNetStepEngine(m, B, L, lr=1e-2, momentum=0.9, use_graph=use_graph)
    eng.set_batch(torch.randn(B, 1, L, device=dev), torch.randint(0, 2, (B,), device=dev))
    for _ in range(warmup):
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng.close()
    return B * steps / dt
