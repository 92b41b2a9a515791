"""Sequence parallelism for long ECG records (SURVEY §5.7 stretch goal; absent from the reference).

The reference only ever sees fixed 500-sample windows (Module_1/shard_prep.py:21-33, win_len=500), so its
"scaling" is batch and world size.  A multi-hour Holter record (~31 M samples per day at 360 Hz) does not fit
that mould: here ONE record is split along time over the ranks of a process group, and every conv layer
exchanges a halo of (K-1) samples with its neighbours over point-to-point sends (RCCL send/recv over xGMI on
MI355X, gloo on CPU), so each rank only ever holds L/world samples of every activation.

Pieces:
  * ``shard_bounds``                contiguous near-equal time shards (the first ``L % world`` get one more).
  * ``halo_exchange``               autograd op: [B,C,l] -> [B,C,left+l+right] with the neighbours' edge samples
                                    (zeros past the record ends = the global zero padding); backward returns the
                                    halo gradients to the ranks that own those samples.
  * ``SeqShardedConv1d``            wraps an ``nn.Conv1d`` (stride 1, dilation 1): halo exchange + valid conv.
  * ``seq_global_avg_pool``         AdaptiveAvgPool1d(1) over the whole record: one all-reduce of [B,C] sums.
  * ``SeqParallelTinyECG``          TinyECG (same parameters / state_dict) over a time-sharded record.
  * ``allreduce_seq_grads_``        after backward: sums the conv parameters' partial gradients over the group
                                    (the head's gradients are already identical everywhere).

Exactness: forward output and all gradients equal the single-process model on the full record up to fp32
summation order (tests/test_seqpar_cpu.py, gloo world 2 and 3).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F


def shard_bounds(L: int, world: int, rank: int) -> Tuple[int, int]:
    """[start, end) of ``rank``'s contiguous time shard of a length-``L`` record."""
    q, r = divmod(L, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def _group_info(group) -> Tuple[int, int]:
    if not (dist.is_available() and dist.is_initialized()):
        return 0, 1
    return dist.get_rank(group), dist.get_world_size(group)


def _global_rank(group, r: int) -> int:
    return r if group is None else dist.get_global_rank(group, r)


def _exchange(send_left: Optional[torch.Tensor], send_right: Optional[torch.Tensor], recv_left_shape, recv_right_shape,
              like: torch.Tensor, group) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
    """Send ``send_left`` to rank-1 and ``send_right`` to rank+1; receive from rank-1 / rank+1 (one batched P2P
    round, so no ordering deadlock).  A ``None`` shape means nothing is expected from that side."""
    rank, world = _group_info(group)
    ops: List[dist.P2POp] = []
    recv_l = recv_r = None
    if rank > 0:
        if recv_left_shape is not None:
            recv_l = torch.empty(recv_left_shape, dtype=like.dtype, device=like.device)
            ops.append(dist.P2POp(dist.irecv, recv_l, _global_rank(group, rank - 1), group))
        if send_left is not None:
            ops.append(dist.P2POp(dist.isend, send_left.contiguous(), _global_rank(group, rank - 1), group))
    if rank < world - 1:
        if send_right is not None:
            ops.append(dist.P2POp(dist.isend, send_right.contiguous(), _global_rank(group, rank + 1), group))
        if recv_right_shape is not None:
            recv_r = torch.empty(recv_right_shape, dtype=like.dtype, device=like.device)
            ops.append(dist.P2POp(dist.irecv, recv_r, _global_rank(group, rank + 1), group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return recv_l, recv_r


class _HaloExchange(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: torch.Tensor, left: int, right: int, group) -> torch.Tensor:
        rank, world = _group_info(group)
        B, C, l = x.shape
        if l < max(left, right):
            raise ValueError(f"time shard of {l} samples is shorter than the conv halo ({left}, {right})")
        ctx.left, ctx.right, ctx.group = left, right, group
        # my head goes to rank-1 (its right halo), my tail to rank+1 (its left halo)
        head = x[..., :right] if right > 0 else None
        tail = x[..., l - left:] if left > 0 else None
        got_l, got_r = _exchange(head, tail, (B, C, left) if left > 0 else None, (B, C, right) if right > 0 else None,
                                 x, group)
        zl = x.new_zeros(B, C, left)
        zr = x.new_zeros(B, C, right)
        return torch.cat([got_l if got_l is not None else zl, x, got_r if got_r is not None else zr], dim=2)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        left, right, group = ctx.left, ctx.right, ctx.group
        B, C, lp = g.shape
        l = lp - left - right
        gx = g[..., left:left + l].clone()
        # gradient of my left halo belongs to rank-1's tail; of my right halo to rank+1's head
        g_left_halo = g[..., :left] if left > 0 else None
        g_right_halo = g[..., left + l:] if right > 0 else None
        from_l, from_r = _exchange(g_left_halo, g_right_halo, (B, C, right) if right > 0 else None,
                                   (B, C, left) if left > 0 else None, g, group)
        # rank-1 sent the gradient of ITS right halo = my head; rank+1 the gradient of its left halo = my tail
        if from_l is not None:
            gx[..., :right] += from_l
        if from_r is not None:
            gx[..., l - left:] += from_r
        return gx, None, None, None


def halo_exchange(x: torch.Tensor, left: int, right: int, group=None) -> torch.Tensor:
    """[B,C,l] time shard -> [B,C,left+l+right] with the neighbouring shards' edge samples (zeros at the record
    ends).  Differentiable: the halo gradients are returned to the owning ranks."""
    _, world = _group_info(group)
    if world == 1:
        return F.pad(x, (left, right))
    return _HaloExchange.apply(x, left, right, group)


class SeqShardedConv1d(nn.Module):
    """``conv`` (stride 1, dilation 1, odd K, zero padding (K-1)/2) applied to a time-sharded signal; shares
    ``conv``'s parameters.  Halo = (K-1)/2 samples on each side."""

    def __init__(self, conv: nn.Conv1d, group=None):
        super().__init__()
        if conv.stride != (1,) or conv.dilation != (1,) or conv.groups != 1 or conv.padding_mode != "zeros":
            raise ValueError("SeqShardedConv1d needs stride 1, dilation 1, groups 1, zero padding")
        if isinstance(conv.padding, str):
            raise ValueError("explicit integer padding required")
        self.conv, self.group = conv, group
        K, p = conv.kernel_size[0], conv.padding[0]
        if 2 * p != K - 1:
            raise ValueError("SeqShardedConv1d needs a length-preserving conv (odd K, padding (K-1)/2)")
        self.left, self.right = p, K - 1 - p

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        xp = halo_exchange(x, self.left, self.right, self.group)
        return F.conv1d(xp, self.conv.weight, self.conv.bias)


class _AllReduceSum(torch.autograd.Function):
    """Forward: sum over the group.  Backward: identity - every rank computes the same downstream loss from the
    same reduced value, so each rank's share already receives the full upstream gradient."""

    @staticmethod
    def forward(ctx, t: torch.Tensor, group) -> torch.Tensor:
        out = t.clone()
        dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        return out

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        return g, None


def seq_global_avg_pool(h: torch.Tensor, L_total: int, group=None) -> torch.Tensor:
    """AdaptiveAvgPool1d(1) + squeeze over the whole record: [B,C,l] local -> [B,C] global mean."""
    s = h.sum(dim=2)
    _, world = _group_info(group)
    if world > 1:
        s = _AllReduceSum.apply(s, group)
    return s / float(L_total)


class SeqParallelTinyECG(nn.Module):
    """TinyECG over a time-sharded record.  Wraps (and shares the parameters of) a ``TinyECG``; input is this
    rank's [B,1,l] shard, output the [B,C] logits of the whole record (identical on every rank)."""

    def __init__(self, model: nn.Module, group=None):
        super().__init__()
        self.model, self.group = model, group
        self.c1 = SeqShardedConv1d(model.net[0], group)
        self.c2 = SeqShardedConv1d(model.net[2], group)

    def forward(self, x_local: torch.Tensor, L_total: int) -> torch.Tensor:
        h = F.relu(self.c1(x_local))
        h = F.relu(self.c2(h))
        return self.model.head(seq_global_avg_pool(h, L_total, self.group))


def seq_sharded_params(model: nn.Module) -> List[nn.Parameter]:
    """Parameters whose gradients are partial per time shard (everything before the global pool)."""
    return [p for n, p in model.named_parameters() if not n.startswith("head.")]


def allreduce_seq_grads_(model: nn.Module, group=None) -> None:
    """Sum the conv parameters' per-shard gradients over the group (one flat all-reduce)."""
    _, world = _group_info(group)
    ps = [p for p in seq_sharded_params(model) if p.grad is not None]
    if world == 1 or not ps:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    o = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[o:o + n].view_as(p.grad))
        o += n
