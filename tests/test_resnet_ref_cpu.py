"""The teacher-forced per-block references (models/resnet1d_ref.py) equal PyTorch autograd of a training-mode
BasicBlock1D in float64 - the oracle the GPU engine test (test_resnet_engine_gpu.py) is pinned against."""
import pytest
import torch
import torch.nn.functional as F

import crossscale_ecg  # noqa: F401
from crossscale_ecg.models.resnet1d import BasicBlock1D
from crossscale_ecg.models.resnet1d_ref import block_backward_reference, block_forward_reference


@pytest.mark.parametrize("cin,cout,stride", [(16, 16, 1), (16, 32, 2)])
def test_block_reference_matches_autograd(cin, cout, stride):
    torch.manual_seed(0)
    blk = BasicBlock1D(cin, cout, stride).double().train()
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.2, 0.2)
    h = F.relu(torch.randn(4, cin, 37, dtype=torch.float64)).requires_grad_(True)
    # module forward with the intermediates exposed
    z1 = blk.conv1(h)
    a1 = F.relu(blk.bn1(z1))
    z2 = blk.conv2(a1)
    zd = blk.downsample[0](h) if blk.downsample is not None else None
    idt = blk.downsample[1](zd) if zd is not None else h
    pre = blk.bn2(z2) + idt
    out = F.relu(pre)
    up = torch.randn_like(out)
    for t in (z1, a1, z2, pre):
        t.retain_grad()
    out.backward(up)
    eps = blk.bn1.eps
    bn = {"bn1": (blk.bn1.weight.detach(), blk.bn1.bias.detach()), "bn2": (blk.bn2.weight.detach(), blk.bn2.bias.detach())}
    Wd = None
    if blk.downsample is not None:
        bn["ds"] = (blk.downsample[1].weight.detach(), blk.downsample[1].bias.detach())
        Wd = blk.downsample[0].weight.detach()
    d = lambda t: None if t is None else t.detach()  # noqa: E731
    fw = block_forward_reference(d(h), d(z1), d(a1), d(z2), d(zd), blk.conv1.weight.detach(),
                                 blk.conv2.weight.detach(), Wd, bn, stride, eps)
    for k, want in (("z1", z1), ("a1", a1), ("z2", z2), ("zd", zd), ("out", out)):
        if want is not None:
            assert torch.allclose(fw[k], want, atol=1e-10), k
    G = pre.grad.detach()
    g, din = block_backward_reference(G, d(h), d(z1), d(a1), d(z2), d(zd), blk.conv1.weight.detach(),
                                      blk.conv2.weight.detach(), Wd, bn, stride, eps, mask_in=False)
    for name, p in blk.named_parameters():
        assert torch.allclose(g[name], p.grad, atol=1e-9, rtol=1e-7), name
    assert torch.allclose(din, h.grad, atol=1e-9)
