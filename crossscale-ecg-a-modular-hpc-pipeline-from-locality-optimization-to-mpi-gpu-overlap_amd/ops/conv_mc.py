"""Multi-channel conv1d on MFMA (csrc/kernels/conv1d_mc.hip) as a differentiable op, channels-last.

``conv1d_nlc(x, weight, bias, stride, padding)``: x [B, L, C_in] bf16 (NLC), weight [C_out, C_in, K] (the
nn.Conv1d parameter, fp32 master), bias [C_out] or None -> y [B, L_out, C_out] bf16.
  forward    = ecg_conv1d_nlc_fwd (implicit GEMM, bias fused)
  grad input = ecg_conv1d_nlc_fwd on dy with input dilation ``stride``, flipped taps, pad K-1-p
  grad weight= ecg_conv1d_nlc_wgrad (split-K fp32 partials, summed in a fixed order -> deterministic)
  grad bias  = sum of dy over (B, L)
Constraints: C_in % 64 == 0 and C_out % 64 == 0 (``supported()``); callers fall back to MIOpen otherwise.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _lib


def supported(c_in: int, c_out: int) -> bool:
    return c_in % 64 == 0 and c_out % 64 == 0


def out_len(L: int, K: int, stride: int, pad: int) -> int:
    return (L + 2 * pad - K) // stride + 1


def _bind(lib):
    if getattr(lib, "_conv_mc_bound", False):
        return
    vp, i32 = _lib.vp, _lib.i32
    _lib._sig(lib, "ecg_conv1d_nlc_fwd", [vp, vp, vp, vp] + [i32] * 10 + [vp])
    _lib._sig(lib, "ecg_conv1d_nlc_wgrad", [vp, vp, vp] + [i32] * 9 + [vp])
    _lib._sig(lib, "ecg_conv1d_nlc_wgrad_tiles", [i32, i32, i32])
    _lib._sig(lib, "ecg_conv1d_nlc_wgrad_target_wgs", [i32] * 6)
    _lib._sig(lib, "ecg_conv1d_nlc_wgrad_splits", [i32] * 8)
    _lib._sig(lib, "ecg_conv1d_nlc_set_big", [i32])
    _lib._sig(lib, "ecg_conv1d_nlc_set_mt", [i32])
    _lib._sig(lib, "ecg_conv1d_nlc_set_tap", [i32])
    _lib._sig(lib, "ecg_conv1d_nlc_set_tap64", [i32])
    _lib._sig(lib, "ecg_conv1d_nlc_set_dma_dil", [i32])
    _lib._sig(lib, "ecg_conv1d_nlc_set_tap_s2", [i32])
    _lib._sig(lib, "ecg_conv1d_nlc_fwd_ex", [vp] * 7 + [i32] * 10 + [vp, vp, vp])
    _lib._sig(lib, "ecg_conv1d_nlc_fwd_stat_tiles", [_lib.C.c_long, i32])
    _lib._sig(lib, "ecg_conv1d_nlc_fwd_stat_rows", [i32] * 9)
    _lib._sig(lib, "ecg_conv1d_nlc_fwd_pa", [vp] * 7 + [i32] * 10 + [vp, vp, vp, vp])
    _lib._sig(lib, "ecg_conv1d_nlc_pa_ok", [i32] * 9)
    lib._conv_mc_bound = True


def _lib_k():
    lib = _lib.kernels()
    _bind(lib)
    return lib


def set_tile_family(big: int) -> int:
    """256-row forward tiles of the LDS-DMA loop (0: 128-row tiles only, 1 (default): + 256x256, 2: + 256x128);
    returns the previous setting.  Step plans built before a change keep the tiling they were built with: set it
    first."""
    return _lib_k().ecg_conv1d_nlc_set_big(int(big))


def set_dma_dilated(on: bool) -> int:
    """Strided (phase-decomposed) data-grads on the LDS-DMA loop (True, default) or the register-staged loop;
    returns the previous setting."""
    return _lib_k().ecg_conv1d_nlc_set_dma_dil(1 if on else 0)


def set_tap_shared(mode: int) -> int:
    """Tap-shared 256-row forward/data-grad kernel for stride-1 pad-1 3-tap convs (0: off, 1 (default): outputs with
    C_out % 128 == 0, 2: also 64-channel outputs); returns the previous mode.  Build step plans after setting it."""
    return _lib_k().ecg_conv1d_nlc_set_tap(int(mode))


def set_tap_s2(on: bool) -> int:
    """Tap-shared strided data-grad kernel (the data-grads of stride-2 pad-1 3-tap convs: one staged dz image per
    chunk read by both output phases) (True, default) or the phase-decomposed one-tap kernels; returns the previous
    setting.  Build step plans after setting it."""
    return _lib_k().ecg_conv1d_nlc_set_tap_s2(1 if on else 0)


def set_tap64(on: bool) -> int:
    """Persistent 64-channel tap kernel (weights resident in LDS, A' images streamed per 128-row tile, one partial
    row per workgroup) for C_in == C_out == 64 stride-1 3-tap convs (True, default) or the one-tap kernels; returns
    the previous setting.  Build step plans after setting it."""
    return _lib_k().ecg_conv1d_nlc_set_tap64(1 if on else 0)


def set_multi_tile(mode: int) -> int:
    """Multi-tile forward workgroups (0: one tile per workgroup, 1 (default): 128x64 tiles of launches with more
    tiles than two resident workgroups per CU, 2: + the 128-channel shapes); returns the previous mode.  Step plans
    size their BatchNorm partial rows when built: set it first."""
    return _lib_k().ecg_conv1d_nlc_set_mt(int(mode))


def stat_rows(B: int, L_in: int, c_in: int, L_out: int, c_out: int, k: int = 3, stride: int = 1, pad: int = 1,
              in_dil: int = 1) -> int:
    """Rows of BatchNorm partials the forward kernel writes for that exact conv (the kernel family - tap-shared,
    multi-tile, one-tile - and its tile size depend on the whole shape, not just M and c_out)."""
    return _lib_k().ecg_conv1d_nlc_fwd_stat_rows(int(B), int(L_in), int(c_in), int(L_out), int(c_out), int(k),
                                                 int(stride), int(pad), int(in_dil))


def fwd_stats_raw(x: torch.Tensor, w_t: torch.Tensor, stride: int, pad: int, L_out: int):
    """Forward conv with the BatchNorm-statistics epilogue (the ResNet plan's CONV_FWD, no fused finalize):
    returns y [B, L_out, Cout] bf16 and the partial rows [2, rows, Cout] fp32 (sum y, sum y^2 of the stored bf16
    values; summed over rows they are the per-channel batch statistics)."""
    B, Lin, Cin = x.shape
    Cout, K, _ = w_t.shape
    if not (x.dtype == w_t.dtype == torch.bfloat16 and x.is_contiguous() and w_t.is_contiguous()):
        raise ValueError("conv1d_nlc: contiguous bf16 operands required")
    rows = _lib_k().ecg_conv1d_nlc_fwd_stat_rows(B, Lin, Cin, L_out, Cout, K, stride, pad, 1)
    y = torch.empty((B, L_out, Cout), dtype=torch.bfloat16, device=x.device)
    stats = torch.empty((2, rows, Cout), dtype=torch.float32, device=x.device)
    st = _lib_k().ecg_conv1d_nlc_fwd_ex(x.data_ptr(), w_t.data_ptr(), None, y.data_ptr(), stats.data_ptr(), None,
                                        None, B, Lin, Cin, L_out, Cout, K, stride, pad, 1, 0, None, None,
                                        _lib.stream_ptr(x.device))
    _lib.check(st, "ecg_conv1d_nlc_fwd_ex")
    return y, stats


def pre_act_ok(B: int, L: int, c_in: int, c_out: int) -> bool:
    """Whether a stride-1 pad-1 3-tap conv over [B, L, c_in] -> c_out takes an input pre-activation (the 128-column
    tap-shared kernel)."""
    return bool(_lib_k().ecg_conv1d_nlc_pa_ok(int(B), int(L), int(c_in), int(L), int(c_out), 3, 1, 1, 1))


def fwd_pre_act_raw(z: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, w_t: torch.Tensor):
    """Stride-1 pad-1 3-tap conv of relu(z * scale + shift) (per input channel: a BatchNorm + ReLU folded into the
    tap-shared kernel's staged operand image).  Returns (y, a) with a the activated operand the kernel stores for the
    weight gradient.  z [B, L, C_in] bf16, scale / shift [C_in] fp32, w_t [C_out, 3, C_in] bf16."""
    B, L, Cin = z.shape
    Cout = w_t.shape[0]
    if not (z.dtype == w_t.dtype == torch.bfloat16 and z.is_contiguous() and w_t.is_contiguous()
            and scale.dtype == shift.dtype == torch.float32 and scale.numel() == shift.numel() == Cin):
        raise ValueError("fwd_pre_act_raw: contiguous bf16 z / w_t and fp32 [C_in] scale / shift required")
    if not pre_act_ok(B, L, Cin, Cout):
        raise ValueError("fwd_pre_act_raw: shape not routed to the tap-shared kernel")
    y = torch.empty((B, L, Cout), dtype=torch.bfloat16, device=z.device)
    a = torch.empty_like(z)
    sc, sh = scale.contiguous(), shift.contiguous()
    pa = (_lib.C.c_void_p * 3)(sc.data_ptr(), sh.data_ptr(), a.data_ptr())
    st = _lib_k().ecg_conv1d_nlc_fwd_pa(z.data_ptr(), w_t.data_ptr(), None, y.data_ptr(), None, None, None, B, L, Cin,
                                        L, Cout, 3, 1, 1, 1, 0, None, None, pa, _lib.stream_ptr(z.device))
    _lib.check(st, "ecg_conv1d_nlc_fwd_pa")
    return y, a


def fwd_raw(x: torch.Tensor, w_t: torch.Tensor, bias: Optional[torch.Tensor], stride: int, pad: int,
            L_out: int, in_dil: int = 1, relu: bool = False) -> torch.Tensor:
    """x [B, Lin, Cin] bf16, w_t [Cout, K, Cin] bf16 -> y [B, L_out, Cout] bf16."""
    B, Lin, Cin = x.shape
    Cout, K, Cin2 = w_t.shape
    if Cin2 != Cin or x.dtype != torch.bfloat16 or w_t.dtype != torch.bfloat16:
        raise ValueError("conv1d_nlc: bf16 x [B,L,Cin] and w [Cout,K,Cin] required")
    if not (x.is_contiguous() and w_t.is_contiguous()):
        raise ValueError("conv1d_nlc: contiguous operands required")
    if not supported(Cin, Cout):
        raise ValueError(f"conv1d_nlc needs C_in, C_out multiples of 64 (got {Cin}, {Cout})")
    y = torch.empty((B, L_out, Cout), dtype=torch.bfloat16, device=x.device)
    b = None if bias is None else bias.float().contiguous()
    st = _lib_k().ecg_conv1d_nlc_fwd(x.data_ptr(), w_t.data_ptr(), _lib.ptr(b), y.data_ptr(), B, Lin, Cin, L_out, Cout,
                                     K, stride, pad, in_dil, int(relu), _lib.stream_ptr(x.device))
    _lib.check(st, "ecg_conv1d_nlc_fwd")
    return y


def wgrad_raw(dy: torch.Tensor, x: torch.Tensor, K: int, stride: int, pad: int,
              splits: Optional[int] = None) -> torch.Tensor:
    """dw [Cout, K, Cin] fp32 from dy [B, Lout, Cout] and x [B, Lin, Cin] (bf16)."""
    B, Lout, Cout = dy.shape
    _, Lin, Cin = x.shape
    R = B * Lout
    chunks = (R + 63) // 64
    lib = _lib_k()
    tiles = lib.ecg_conv1d_nlc_wgrad_tiles(Cout, K, Cin)
    if splits is None:  # the tap-shared kernel's plan, else: target workgroups, >= 8 chunks each, <= 256 slices
        splits = lib.ecg_conv1d_nlc_wgrad_splits(B, Lin, Cin, Lout, Cout, K, stride, pad)
    if not splits:
        target = lib.ecg_conv1d_nlc_wgrad_target_wgs(Cout, K, Cin, B, Lin, Lout)
        splits = max(1, min(256, max(1, chunks // 8), max(1, target // max(1, tiles))))
    part = torch.empty((splits, Cout, K * Cin), dtype=torch.float32, device=dy.device)
    st = _lib_k().ecg_conv1d_nlc_wgrad(dy.data_ptr(), x.data_ptr(), part.data_ptr(), splits, B, Lin, Cin, Lout, Cout, K,
                                       stride, pad, _lib.stream_ptr(dy.device))
    _lib.check(st, "ecg_conv1d_nlc_wgrad")
    return part.sum(0).view(Cout, K, Cin)


class Conv1dNLC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride: int, pad: int):
        Cout, Cin, K = weight.shape
        L_out = out_len(x.shape[1], K, stride, pad)
        w_t = weight.detach().permute(0, 2, 1).to(torch.bfloat16).contiguous()  # [Cout, K, Cin]
        xb = x.to(torch.bfloat16).contiguous()
        y = fwd_raw(xb, w_t, bias.detach() if bias is not None else None, stride, pad, L_out)
        ctx.save_for_backward(xb, weight)
        ctx.has_bias = bias is not None
        ctx.stride, ctx.pad = stride, pad
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, weight = ctx.saved_tensors
        Cout, Cin, K = weight.shape
        dyb = dy.to(torch.bfloat16).contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # dx[u] = sum_k' w[K-1-k'] * dil_s(dy)[u + k' - (K-1-p)]
            w_d = weight.detach().flip(2).permute(1, 2, 0).to(torch.bfloat16).contiguous()  # [Cin, K, Cout]
            dx = fwd_raw(dyb, w_d, None, 1, K - 1 - ctx.pad, xb.shape[1], in_dil=ctx.stride)
        if ctx.needs_input_grad[1]:
            dw = wgrad_raw(dyb, xb, K, ctx.stride, ctx.pad).permute(0, 2, 1).contiguous().to(weight.dtype)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.float().sum(dim=(0, 1)).to(weight.dtype)
        return dx, dw, db, None, None


def conv1d_nlc(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, stride: int = 1,
               padding: int = 0) -> torch.Tensor:
    if padding > weight.shape[2] - 1:
        raise ValueError("padding must be < kernel size (data-grad uses pad K-1-p)")
    return Conv1dNLC.apply(x, weight, bias, stride, padding)
