#!/usr/bin/env python3
"""Timing ablation of the two-launch TinyECG round graph (results are wrong by construction, timing only):
per-step graph time with the real kernels, with the slab reduction replaced by an empty kernel of the same grid,
with the step kernel replaced, and with both (ECG_TINY_ABLATE, read once per process -> one process per mode)."""
import os
import subprocess
import sys

CODE = r'''
import os, sys, torch
sys.path.insert(0, os.getcwd())
import crossscale_ecg
from crossscale_ecg.models.tiny_ecg import TinyECG
from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
dev = torch.device("cuda:0")
x = torch.randn(20000, 500, device=dev); y = torch.zeros(20000, dtype=torch.long, device=dev)
tr = FusedTinyTrainer(TinyECG().to(dev), x, y, 256, 50, seed=0, persistent=False)
for _ in range(5): tr.run_round()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): tr.run_round()
e1.record(); torch.cuda.synchronize()
print(f"{os.environ.get('ECG_TINY_ABLATE', 'none'):7s}: {e0.elapsed_time(e1) * 1e3 / (20 * 50):.3f} us/step", flush=True)
'''

for mode in ("none", "reduce", "step", "both"):
    env = dict(os.environ)
    if mode != "none":
        env["ECG_TINY_ABLATE"] = mode
    subprocess.run([sys.executable, "-c", CODE], env=env, check=True)
