#!/usr/bin/env python3
"""Trace the pseudo-FL G1 step (``train.pseudo_fl.run_overlap_gpu``) to explain its per-step time.

Round 1 recorded G1_overlap_amp at 20.6 ms/step against ~3 ms for the same eager bf16 step elsewhere.  This
runs G0, G1 and a plain eager bf16 step (no side stream) for a few steps each under ``torch.profiler`` and
prints the top host/device ops, so the extra time is attributed rather than re-measured.
"""
from __future__ import annotations

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.data.dataset import make_gpu_batch_iter  # noqa: E402
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.train.pseudo_fl import run_baseline_gpu, run_overlap_gpu  # noqa: E402


def plain_bf16(model, it, dev, steps):
    model = model.to(dev)
    opt = torch.optim.SGD(model.parameters(), lr=1e-2, momentum=0.9)
    for i in range(steps + 5):
        if i == 5:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        x, y = next(it)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def main():
    dev = torch.device("cuda:0")
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag_g1"
    os.makedirs(out, exist_ok=True)
    g = torch.Generator(device=dev)
    g.manual_seed(1337)
    x = torch.randn(20000, 500, generator=g, device=dev)
    y = torch.zeros(20000, dtype=torch.long, device=dev)
    B, steps = 256, 50
    lines = []
    torch.manual_seed(0)
    st = run_baseline_gpu(TinyECG(), make_gpu_batch_iter(x, y, B), dev, steps, 0, B, log_every=0)
    lines.append(f"G0 step_ms {st.step_ms:.3f} compute_ms {st.compute_ms:.3f} data_ms {st.data_ms:.3f}")
    torch.manual_seed(0)
    st = run_overlap_gpu(TinyECG(), make_gpu_batch_iter(x, y, B), dev, steps, 0, B, log_every=0)
    lines.append(f"G1 step_ms {st.step_ms:.3f} compute_ms {st.compute_ms:.3f} data_ms {st.data_ms:.3f}")
    torch.manual_seed(0)
    lines.append(f"plain bf16 (same process, no side stream) step_ms {plain_bf16(TinyECG(), make_gpu_batch_iter(x, y, B), dev, steps):.3f}")
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    for name, fn in (("G1", lambda: run_overlap_gpu(TinyECG(), make_gpu_batch_iter(x, y, B), dev, 10, 0, B,
                                                    log_every=0, warmup=2)),
                     ("G0", lambda: run_baseline_gpu(TinyECG(), make_gpu_batch_iter(x, y, B), dev, 10, 0, B,
                                                     log_every=0, warmup=2))):
        with torch.profiler.profile(activities=acts) as prof:
            fn()
        tab = prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25)
        tab2 = prof.key_averages().table(sort_by="self_device_time_total", row_limit=25)
        with open(os.path.join(out, f"{name}_profile.txt"), "w") as f:
            f.write(tab + "\n\n" + tab2 + "\n")
        prof.export_chrome_trace(os.path.join(out, f"{name}_trace.json"))
    with open(os.path.join(out, "summary.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
