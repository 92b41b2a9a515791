"""bf16-emulating fp64 reference of the native ResNet1D step engine (numerics oracle for the HIP engine).

The engine (ops/resnet_engine.py, csrc/kernels/resnet_nlc.hip + conv1d_mc.hip) keeps fp32 master weights but
stores every activation and every activation gradient in bf16 and feeds bf16 weights to its MFMA convs.  A
plain fp32 (or autocast) PyTorch model rounds at different points, and a deep random-init ResNet amplifies those
rounding differences chaotically (round 1 had to accept 100 % per-tensor gradient error at depth 34).  This
reference runs in float64 and rounds to bf16 exactly where the engine stores bf16:

* forward  ``Q`` (round to bf16; gradient rounded to bf16 on the way back) on z0 (stem conv out), h0 (stem
  BN+ReLU+pool out), and per block on z1, a1 = ReLU(BN1(z1)), z2, zd (downsample conv out) and the block
  output; ``W`` (round, identity gradient) on every block conv weight;
* backward therefore rounds d(out), d(z2), d(a1), d(z1), d(zd), d(h0) - the engine's bf16 gradient buffers;
* everything else (BN statistics and apply, pooling, head, softmax-CE, weight-gradient accumulation) in fp64.

What is left between engine and reference is fp32-vs-fp64 accumulation order and the values that land on the
other side of a bf16 rounding boundary because of it.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.nn.functional as F

from .resnet1d import ResNet1D


class _Q(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).to(g.dtype)


class _W(torch.autograd.Function):
    @staticmethod
    def forward(ctx, w):
        return w.to(torch.bfloat16).to(w.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


def _bn_p(x, bn, params, pre):
    """Training-mode BatchNorm1d over (N, L) in fp64 (biased variance), affine from ``params``."""
    mean = x.mean(dim=(0, 2), keepdim=True)
    var = ((x - mean) ** 2).mean(dim=(0, 2), keepdim=True)
    return (x - mean) * torch.rsqrt(var + bn.eps) * params[pre + "weight"].view(1, -1, 1) + \
        params[pre + "bias"].view(1, -1, 1)


def reference_grads(model: ResNet1D, x: torch.Tensor, y: torch.Tensor) -> Tuple[float, Dict[str, torch.Tensor]]:
    """(loss, {name: grad}) of the bf16-emulating fp64 reference for the model's current parameters."""
    params = {n: p.detach().to(torch.float64).clone().requires_grad_(True) for n, p in model.named_parameters()}
    Q = _Q.apply
    xx = x.to(torch.float64)
    z0 = Q(F.conv1d(xx, params["conv1.weight"], None, model.conv1.stride, model.conv1.padding))
    h = Q(F.max_pool1d(F.relu(_bn_p(z0, model.bn1, params, "bn1.")), 3, 2, 1))
    W = _W.apply
    for si, stage in enumerate((model.layer1, model.layer2, model.layer3, model.layer4)):
        for bi, blk in enumerate(stage):
            pre = f"layer{si + 1}.{bi}."
            z1 = Q(F.conv1d(h, W(params[pre + "conv1.weight"]), None, blk.conv1.stride, 1))
            a1 = Q(F.relu(_bn_p(z1, blk.bn1, params, pre + "bn1.")))
            z2 = Q(F.conv1d(a1, W(params[pre + "conv2.weight"]), None, 1, 1))
            if blk.downsample is not None:
                zd = Q(F.conv1d(h, W(params[pre + "downsample.0.weight"]), None, blk.downsample[0].stride, 0))
                idt = _bn_p(zd, blk.downsample[1], params, pre + "downsample.1.")
            else:
                idt = h
            h = Q(F.relu(_bn_p(z2, blk.bn2, params, pre + "bn2.") + idt))
    feat = h.mean(dim=2)
    logits = F.linear(feat, params["fc.weight"], params["fc.bias"])
    loss = F.cross_entropy(logits, y)
    loss.backward()
    return float(loss.detach()), {n: p.grad.detach() for n, p in params.items()}


# ------------------------------------------------------------------------------------------------------------
# Teacher-forced per-block references.  End-to-end gradients of a deep random-init net are chaotic under bf16
# (above: the emulated reference itself is 45-80 % off fp64 at depth 18/34), so the engine is pinned op by op
# instead: every block's forward is recomputed in fp64 from the ENGINE's own input activation, and every
# block's backward from the engine's own incoming gradient and saved activations.  The remaining difference
# is the engine's bf16 storage of the block's outputs / intermediate gradients and fp32 accumulation order.
# All tensors NCL float64; weights as the engine sees them (bf16-rounded) are passed in.

def bn_batch_stats(z: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Training-mode BatchNorm statistics over (N, L): per-channel mean and biased variance (keepdim)."""
    mean = z.mean(dim=(0, 2), keepdim=True)
    var = ((z - mean) ** 2).mean(dim=(0, 2), keepdim=True)
    return mean, var


def bn_apply(z, gamma, beta, eps):
    mean, var = bn_batch_stats(z)
    return (z - mean) * torch.rsqrt(var + eps) * gamma.view(1, -1, 1) + beta.view(1, -1, 1)


def bn_backward(dy, z, gamma, eps):
    """(dz, dgamma, dbeta) of y = BN(z) (training mode) for upstream gradient dy."""
    mean, var = bn_batch_stats(z)
    rstd = torch.rsqrt(var + eps)
    xhat = (z - mean) * rstd
    dbeta = dy.sum(dim=(0, 2))
    dgamma = (dy * xhat).sum(dim=(0, 2))
    n = z.shape[0] * z.shape[2]
    dz = gamma.view(1, -1, 1) * rstd * (dy - dbeta.view(1, -1, 1) / n - xhat * dgamma.view(1, -1, 1) / n)
    return dz, dgamma, dbeta


def block_forward_reference(h, z1, a1, z2, zd, W1, W2, Wd, bn, stride, eps):
    """Per-op forward references of a BasicBlock, each from the engine's own previous-op output:
    {z1, a1, z2, zd, out} computed from (h | z1 | a1 | h | z2, zd) respectively.  ``bn``: dict of
    (gamma, beta) for keys 'bn1', 'bn2' and 'ds' (when Wd is given)."""
    out = {"z1": F.conv1d(h, W1, None, stride, 1)}
    out["a1"] = F.relu(bn_apply(z1, *bn["bn1"], eps))
    out["z2"] = F.conv1d(a1, W2, None, 1, 1)
    idt = h
    if Wd is not None:
        out["zd"] = F.conv1d(h, Wd, None, stride, 0)
        idt = bn_apply(zd, *bn["ds"], eps)
    out["out"] = F.relu(bn_apply(z2, *bn["bn2"], eps) + idt)
    return out


def block_backward_reference(G, h, z1, a1, z2, zd, W1, W2, Wd, bn, stride, eps, mask_in: bool):
    """Backward of a BasicBlock from G = dL/d(BN2(z2) + identity) (already ReLU-masked by the block's output
    ReLU), every step on the engine's saved activations.  Returns parameter gradients and d(input)
    (times relu'(h) when ``mask_in``: the previous block's output ReLU, as the engine stores it)."""
    g = {}
    dz2, g["bn2.weight"], g["bn2.bias"] = bn_backward(G, z2, bn["bn2"][0], eps)
    g["conv2.weight"] = torch.nn.grad.conv1d_weight(a1, W2.shape, dz2, 1, 1)
    da1 = torch.nn.grad.conv1d_input(a1.shape, W2, dz2, 1, 1) * (a1 > 0)
    dz1, g["bn1.weight"], g["bn1.bias"] = bn_backward(da1, z1, bn["bn1"][0], eps)
    g["conv1.weight"] = torch.nn.grad.conv1d_weight(h, W1.shape, dz1, stride, 1)
    din = torch.nn.grad.conv1d_input(h.shape, W1, dz1, stride, 1)
    if Wd is not None:
        dzd, g["downsample.1.weight"], g["downsample.1.bias"] = bn_backward(G, zd, bn["ds"][0], eps)
        g["downsample.0.weight"] = torch.nn.grad.conv1d_weight(h, Wd.shape, dzd, stride, 0)
        din = din + torch.nn.grad.conv1d_input(h.shape, Wd, dzd, stride, 0)
    else:
        din = din + G
    if mask_in:
        din = din * (h > 0)
    return g, din
