"""Diagnostic: ResNet1D-18 B=64 single-batch SGD progress (the test_engine_sgd_step_and_training_progress setup)
under one plan-knob setting (environment), plus the engine gradient vs fp32 torch per parameter."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crossscale_ecg  # noqa: F401
from crossscale_ecg.models.resnet1d import resnet1d18, resnet1d34
from crossscale_ecg.ops.resnet_engine import ResNetStepEngine

DEV = "cuda:0"
depth = int(sys.argv[1]) if len(sys.argv) > 1 else 18
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
torch.manual_seed(0)
m = (resnet1d18 if depth == 18 else resnet1d34)().to(DEV)
ref = copy.deepcopy(m)
x = torch.randn(B, 1, 500, device=DEV)
y = torch.randint(0, 2, (B,), device=DEV)
eng = ResNetStepEngine(m, B, 500, lr=0.05, momentum=0.9)
eng.set_batch(x, y)
eng.forward_backward()
torch.cuda.synchronize()
ref.zero_grad(set_to_none=True)
loss = F.cross_entropy(ref(x), y)
loss.backward()
worst = []
for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
    gi = p.grad
    e = (gi.float().reshape(-1) - q.grad.float().reshape(-1)).norm().item() / (q.grad.norm().item() + 1e-12)
    worst.append((e, n))
worst.sort(reverse=True)
print("knobs", {k: v for k, v in os.environ.items() if k.startswith("ECG_")})
print("loss eng %.5f torch %.5f" % (eng.avg_loss(), loss.item()))
print("worst grad rel err", [(n, round(e, 4)) for e, n in worst[:6]])
eng.reset_loss()
losses = []
for _ in range(30):
    eng.step()
    losses.append(round(eng.avg_loss(), 4))
    eng.reset_loss()
print("losses", losses)
