"""Native ResNet1D training step: the whole forward + backward + SGD step as ONE encoded launch plan
(csrc/kernels/resnet_nlc.hip), replayed eagerly by the C++ plan executor or captured into a single hipGraph.

BASELINE.json config 5 (ResNet1D-34 stress, bf16, large batch).  Design (MI355X-first, see the .hip header):

* one flat fp32 buffer holds every parameter (then the BN running statistics) - ``parallel.flat`` - so FedAvg
  is one RCCL all-reduce, DDP one bucketed all-reduce per backward segment, SGD one kernel;
* activations are channels-last bf16 ``[B, L, C]`` resident in HBM for the whole step (no NCL<->NLC
  transposes, no MIOpen), all shapes fixed at construction so every pointer is baked into the plan;
* every conv is an MFMA implicit GEMM (conv1d_mc.hip) whose epilogue also emits the BatchNorm statistics;
  BN apply / backward passes are fused with ReLU and the residual;
* backward is laid out in ``segments`` = gradient buckets of ~``bucket_mb`` (default 4 MB, closed at block
  boundaries; layer1 joins the stem's).  The gradients of a segment form one contiguous range of the flat grad
  buffer, so each range is all-reduced on a comm stream while the next segment runs (``run_segments``: the DDP
  overlap of SURVEY §2.4 M5 / §7 step 8).

The reference has no ResNet; parity is against PyTorch's own fp32 ResNet1D (tests/test_resnet_engine_gpu.py).
"""
from __future__ import annotations

import ctypes
import math
import os
import struct
from typing import Callable, Dict, List, Optional, Tuple

import torch

from . import _lib
from ..models.resnet1d import ResNet1D

OP_WORDS = 32
OP = dict(CONV_FWD=1, CONV_WGRAD=2, REDUCE_WGRAD=3, BN_FIN=4, BN_ACT=5, BN_BWD_REDUCE=6, BN_BWD_APPLY=7,
          STEM_FWD=8, STEM_POOL=9, STEM_BWD_REDUCE=10, STEM_WGRAD=11, REDUCE_SUM=12, WEIGHT_PREP=13, HEAD=14,
          HEAD_REDUCE=15, SGD=16, GATHER=17, COUNTER_INC=18)


def _f(x: float) -> int:
    return struct.unpack("<q", struct.pack("<d", float(x)))[0]


def _bind(lib):
    if getattr(lib, "_plan_bound", False):
        return
    vp, i32 = _lib.vp, _lib.i32
    _lib._sig(lib, "ecg_plan_run", [vp, i32, ctypes.POINTER(ctypes.c_int), vp])
    _lib._sig(lib, "ecg_plan_run_ex", [vp, i32, ctypes.POINTER(ctypes.c_int), vp, i32, ctypes.POINTER(ctypes.c_void_p)])
    _lib._sig(lib, "ecg_plan_join", [vp])
    _lib._sig(lib, "ecg_plan_graph_create", [ctypes.POINTER(ctypes.c_void_p), vp, i32, ctypes.POINTER(ctypes.c_int)])
    _lib._sig(lib, "ecg_plan_graph_launch", [vp, vp])
    _lib._sig(lib, "ecg_plan_graph_destroy", [vp])
    _lib._sig(lib, "ecg_plan_op_words", [])
    _lib._sig(lib, "ecg_plan_wentry_bytes", [])
    _lib._sig(lib, "ecg_plan_stem_rows", [])
    _lib._sig(lib, "ecg_conv1d_nlc_fwd_stat_tiles", [ctypes.c_long, i32])
    _lib._sig(lib, "ecg_conv1d_nlc_wgrad_tiles", [i32, i32, i32])
    _lib._sig(lib, "ecg_conv1d_nlc_wgrad_target_wgs", [i32] * 6)
    _lib._sig(lib, "ecg_conv1d_nlc_wgrad_splits", [i32] * 8)
    _lib._sig(lib, "ecg_conv1d_nlc_fwd_stat_tiles_ex", [i32, i32, i32, i32])
    _lib._sig(lib, "ecg_conv1d_nlc_fwd_stat_rows", [i32] * 9)
    _lib._sig(lib, "ecg_conv1d_nlc_pa_ok", [i32] * 9)
    lib._plan_bound = True
    if lib.ecg_plan_op_words() != OP_WORDS or lib.ecg_plan_wentry_bytes() != 40:
        raise _lib.NativeError("resnet plan ABI mismatch (rebuild csrc)")


def _out_len(L: int, K: int, s: int, p: int) -> int:
    return (L + 2 * p - K) // s + 1


class _BN:
    """Per-BatchNorm device state: saved mean / rstd / scale / shift (fwd) and c1 / c2 (bwd)."""

    def __init__(self, bn: torch.nn.BatchNorm1d, dev):
        C = bn.num_features
        self.bn, self.C = bn, C
        self.buf = torch.zeros(6, C, dtype=torch.float32, device=dev)
        self.mean, self.rstd, self.scale, self.shift, self.c1, self.c2 = (self.buf[i] for i in range(6))


class ResNetStepEngine:
    """Fixed-shape training step for a :class:`ResNet1D` (any depth, BasicBlocks, channels multiple of 64).

    ``set_batch(x, y)`` copies a batch into the static input buffers; ``step()`` runs forward, backward and
    SGD; ``forward_backward()`` skips the SGD (tests, DDP) and ``apply_update()`` runs it.
    ``grad_sync(flat_range_tensor)`` - if given - is called for each backward segment's gradient range in
    order (DDP all-reduce hook).  ``source=(X [N, L] fp32, Y [N] int32, table [S, B] int32)`` puts the batch
    gather inside the step plan: step ``c`` of a round reads ``table[c % S]`` (device counter, reset by
    ``reset_counter()``), so one captured step graph serves every batch.
    """

    def __init__(self, model: ResNet1D, batch_size: int, seq_len: int = 500, lr: float = 1e-2,
                 momentum: float = 0.9, weight_decay: float = 0.0, nesterov: bool = False, use_graph: bool = True,
                 grad_sync: Optional[Callable[[torch.Tensor], None]] = None,
                 source: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None,
                 bucket_mb: Optional[float] = None):
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("ResNetStepEngine needs a GPU (HIP kernels)")
        self.lib = _lib.kernels()
        _bind(self.lib)
        self.model, self.dev, self.B, self.L = model, dev, int(batch_size), int(seq_len)
        self.lr, self.momentum, self.wd, self.nesterov = lr, momentum, weight_decay, nesterov
        self.use_graph, self.grad_sync = use_graph, grad_sync
        if model._space is None:
            model.flatten_parameters()
        self.space = model._space
        self.flat = self.space.flat
        self.grad = self.space.grad_buffer()
        self.mom = torch.zeros_like(self.grad)
        self.loss_acc = torch.zeros(1, dtype=torch.float32, device=dev)
        self.counter = torch.zeros(1, dtype=torch.int32, device=dev)
        self.source = source
        if source is not None:
            X, Y, table = source
            if (X.dtype != torch.float32 or X.dim() != 2 or X.shape[1] != seq_len or X.stride(1) != 1
                    or Y.dtype != torch.int32 or table.dtype != torch.int32 or table.dim() != 2
                    or table.shape[1] != batch_size or not table.is_contiguous()):
                raise ValueError("source must be (X fp32 [N, L], Y int32 [N], table int32 [S, B])")
        self._steps_since_sync = 0
        self._loss_steps = 0
        self._keep: List[torch.Tensor] = []
        self._graphs: Dict[str, int] = {}
        self._range_ops: Dict[Tuple[int, int], torch.Tensor] = {}
        # gradient buckets: the backward closes a segment after the first block at which the
        # segment's gradients reach bucket_mb (fp32 bytes), so the first collective starts after layer4's first
        # block instead of after the whole stage; 0 = one segment per stage (round 2's plan)
        if bucket_mb is None:
            bucket_mb = float(os.environ.get("ECG_RESNET_BUCKET_MB", "4"))
        self.bucket_bytes = int(float(bucket_mb) * (1 << 20))
        self._build()

    # ------------------------------------------------------------------------------------------ allocation
    def _t(self, *shape, dtype=torch.bfloat16) -> torch.Tensor:
        t = torch.empty(*shape, dtype=dtype, device=self.dev)
        self._keep.append(t)
        return t

    def _gptr(self, p: torch.Tensor) -> int:
        """Address of parameter ``p``'s gradient inside the flat grad buffer."""
        return self.grad.data_ptr() + 4 * self.space.offset_of(p)

    # ------------------------------------------------------------------------------------------ plan build
    def _build(self):
        m, B, L, dev = self.model, self.B, self.L, self.dev
        c0 = m.conv1
        if c0.in_channels != 1 or c0.out_channels != 64 or c0.kernel_size[0] > 8:
            raise ValueError("engine stem expects Conv1d(1, 64, k<=8)")
        blocks = [blk for st in (m.layer1, m.layer2, m.layer3, m.layer4) for blk in st]
        Ks, Ss, Ps = c0.kernel_size[0], c0.stride[0], c0.padding[0]
        Lz = _out_len(L, Ks, Ss, Ps)
        mp = m.maxpool
        if (mp.kernel_size, mp.stride, mp.padding) != (3, 2, 1):
            raise ValueError("engine stem expects MaxPool1d(3, 2, 1)")
        Lp = _out_len(Lz, 3, 2, 1)
        self.Lz, self.Lp = Lz, Lp

        # ---- shapes per block
        shapes = []
        Lc, Cc = Lp, 64
        for blk in blocks:
            s = blk.conv1.stride[0]
            Co = blk.conv1.out_channels
            if Cc % 64 or Co % 64:
                raise ValueError("engine convs need channels % 64 == 0")
            Lo = _out_len(Lc, 3, s, 1)
            shapes.append((Lc, Cc, Lo, Co, s))
            Lc, Cc = Lo, Co
        self.Lf, self.Cf = Lc, Cc
        ncls = m.fc.out_features
        maxel = max([B * Lz * 64] + [B * max(a[0] * a[1], a[2] * a[3]) for a in shapes])

        # ---- static inputs and activations
        self.x = self._t(B, L, dtype=torch.float32)
        self.y = self._t(B, dtype=torch.int32)
        self.z0 = self._t(B, Lz, 64)
        # the stem max-pool's argmax per output (0..2 within its window), written by the forward for the backward
        self.pool_am = torch.zeros(B * Lp * 64, dtype=torch.uint8, device=dev)
        self.h0 = self._t(B, Lp, 64)
        acts = []
        for (Li, Ci, Lo, Co, s), blk in zip(shapes, blocks):
            a = dict(z1=self._t(B, Lo, Co), a1=self._t(B, Lo, Co), z2=self._t(B, Lo, Co), out=self._t(B, Lo, Co),
                     mb=self._t(B * Lo * Co // 8, dtype=torch.uint8))  # out's ReLU mask, one bit per element
            if blk.downsample is not None:
                a["zd"] = self._t(B, Lo, Co)
            acts.append(a)
        # backward scratch (reused block to block: the plan is stream-ordered)
        gA, gB = self._t(maxel), self._t(maxel)  # ping-pong: grad wrt block output / block input
        dz2, ga1, dz1, dzd, tmp = (self._t(maxel) for _ in range(5))
        # weight gradients on a side stream (csrc/kernels/resnet_nlc.hip, OP_LANE): the BN-backward outputs they
        # read (dz2, dz1, dzd) get one buffer per block instead of block-to-block reuse, and their split-K
        # partials a workspace of their own.  ECG_RESNET_SIDE=0: one stream, as captured before.
        side = os.environ.get("ECG_RESNET_SIDE", "1") != "0"
        self.side_lane = side
        dz0 = self._t(B, Lz, 64)
        # BN states
        bn0 = _BN(m.bn1, dev)
        bns = [(_BN(b.bn1, dev), _BN(b.bn2, dev), _BN(b.downsample[1], dev) if b.downsample is not None else None)
               for b in blocks]
        self._bn_states = [bn0] + [x for t in bns for x in t if x is not None]
        # stats / partial buffers (stream-ordered reuse)
        max_T = max((B * Lz + 63) // 64, max((B * a[2] + 63) // 64 for a in shapes))
        stats = self._t(2 * max_T * 512, dtype=torch.float32)
        chunk_for = lambda C: (256 // (C // 8)) * 16  # noqa: E731  rows per reduce block
        stem_chunk_b = 128  # rows per block of the stem backward (more, shorter blocks than chunk_for(64))
        max_Tb = max((B * Lz + stem_chunk_b - 1) // stem_chunk_b,
                     max((B * a[2] + chunk_for(a[3]) - 1) // chunk_for(a[3]) for a in shapes))
        bpart = self._t(3 * max_Tb * 512, dtype=torch.float32)
        fin_scratch = self._t(1024 * 2 * 512, dtype=torch.float64)
        tickets = torch.zeros(64, dtype=torch.int32, device=dev)
        self._keep.append(tickets)

        # ---- wgrad split plan + workspace
        def wsplits(R, Cout, K, Cin, s=1, Lin=None, Lout=None):
            # stride-1 3-tap convs: the tap-shared kernel's own plan (conv1d_mc.hip, ecg_conv1d_nlc_wgrad_splits)
            if Lout is not None:
                ts = self.lib.ecg_conv1d_nlc_wgrad_splits(B, Lin, Cin, Lout, Cout, K, s, 1 if K == 3 else 0)
                if ts > 0:
                    return ts
            # the kernel's target workgroup count, >= 8 row chunks each, <= 256 partial slices (the reduce reads
            # S x |dW|)
            chunks = (R + 63) // 64
            tiles = self.lib.ecg_conv1d_nlc_wgrad_tiles(Cout, K, Cin)
            target = self.lib.ecg_conv1d_nlc_wgrad_target_wgs(Cout, K, Cin, B, Lin or 0, Lout or 0)
            # cap (ECG_WGRAD_SPLIT_CAP): fewer splits shrink the reduce (S x |dW|) but starve the wgrad kernel of
            # workgroups (round 2: cap 16 -> 5.86, cap 8 -> 7.66 ms/step vs 4.61 uncapped, profiles/r2/
            # resnet_conv_ab.txt); round 6 at target 224: 96 -0.3 % vs 64 on two boxes, 24-48 slower
            # (profiles/r6/wgrad_target_ab.txt)
            cap = int(os.environ.get("ECG_WGRAD_SPLIT_CAP", "96"))
            return max(1, min(cap, 256, max(1, chunks // 8), max(1, target // tiles)))

        ws_need = 0
        for (Li, Ci, Lo, Co, s), blk in zip(shapes, blocks):
            R = B * Lo
            ws_need = max(ws_need, wsplits(R, Co, 3, Ci, s, Li, Lo) * Co * 3 * Ci,
                          wsplits(R, Co, 3, Co, 1, Lo, Lo) * Co * 3 * Co)
            if blk.downsample is not None:
                ws_need = max(ws_need, wsplits(R, Co, 1, Ci) * Co * Ci)
        stem_chunk = max(256, -(-(B * Lz) // 1024))  # <= ~1024 partial slices
        stem_blocks = (B * Lz + stem_chunk - 1) // stem_chunk
        Gb = max(1, min(64, B // 64))
        ws_need = max(ws_need, stem_blocks * 64 * Ks, Gb * (ncls * self.Cf + ncls + 1))
        ws = self._t(ws_need, dtype=torch.float32)
        ws_w = self._t(ws_need, dtype=torch.float32) if side else ws

        # ---- bf16 weight arena (fwd + flipped dgrad layouts) and prep table
        convs = []
        for blk in blocks:
            convs += [blk.conv1, blk.conv2] + ([blk.downsample[0]] if blk.downsample is not None else [])
        total = sum(c.weight.numel() for c in convs)
        self.warena = self._t(2 * total)
        entries, off, block0 = [], 0, 0
        self._wf, self._wb = {}, {}
        for c in convs:
            n = c.weight.numel()
            self._wf[id(c)] = self.warena.data_ptr() + 2 * off
            self._wb[id(c)] = self.warena.data_ptr() + 2 * (total + off)
            entries.append(struct.pack("<qqqiiii", self.space.offset_of(c.weight), off, total + off, c.out_channels,
                                       c.in_channels, c.kernel_size[0], block0))
            off += n
            if c.out_channels % 64 or c.in_channels % 64 or c.kernel_size[0] > 3:
                raise ValueError("weight prep tiles need channels % 64 == 0 and k <= 3")
            block0 += (c.out_channels // 64) * (c.in_channels // 64)  # one 64x64 tile per workgroup
        tab = torch.tensor(list(b"".join(entries)), dtype=torch.uint8).to(dev)
        self._keep.append(tab)
        wprep_blocks = block0

        ops: List[List[int]] = []
        self._segments: List[Tuple[int, int, int, int]] = []  # (op_begin, op_end, grad_lo, grad_hi) elements

        def op(kind, *args, lane=0):
            w = [OP[kind]] + [int(a) for a in args]
            assert len(w) < OP_WORDS, kind  # the last word is the lane (0 main, 1 side, 2 main after a join)
            ops.append(w + [0] * (OP_WORDS - 1 - len(w)) + [lane if side else 0])

        P = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        eps, bnm = m.bn1.eps, (m.bn1.momentum if m.bn1.momentum is not None else 0.1)

        def fin_fwd(st: _BN, T, n):
            G = max(1, min(128, T // 64))
            bn = st.bn
            op("BN_FIN", stats.data_ptr(), stats.data_ptr() + 4 * T * st.C, T, st.C, 0, P(fin_scratch),
               P(tickets), _f(n), _f(eps), _f(bnm), P(bn.weight), P(bn.bias), P(st.mean), P(st.rstd), P(st.scale),
               P(st.shift), P(bn.running_mean), P(bn.running_var), 0, 0, 0, 0, G)

        def fin_bwd(st: _BN, T, n, statB, base=None):
            G = max(1, min(128, T // 64))
            bn = st.bn
            base = bpart.data_ptr() if base is None else base
            op("BN_FIN", base, base + 4 * statB * T * st.C, T, st.C, 1, P(fin_scratch),
               P(tickets), _f(n), _f(eps), _f(bnm), P(bn.weight), P(bn.bias), 0, 0, 0, 0, 0, 0,
               self._gptr(bn.weight), self._gptr(bn.bias), P(st.c1), P(st.c2), G)

        # ---- BatchNorm finalize fused into the statistics-producing conv (csrc/include/bn_tail.h): replaces the
        # BN_FIN op after each conv forward and data-grad conv.  ECG_BN_TAIL=0: separate (one-launch) BN_FIN ops.
        use_tail = os.environ.get("ECG_BN_TAIL", "1") != "0"
        self.bn_tail = use_tail
        tail_blobs: List[bytes] = []
        tails_dev = self._t(160 * 304, dtype=torch.uint8)  # room for 160 fused finalizes (ResNet-34 uses 68)

        def fin_fwd_words(st: _BN, n):
            bn = st.bn
            return struct.pack("<qqddd12q", 0, 1, float(n), eps, bnm, P(bn.weight), P(bn.bias), P(st.mean),
                               P(st.rstd), P(st.scale), P(st.shift), P(bn.running_mean), P(bn.running_var), 0, 0, 0, 0)

        def fin_bwd_words(st: _BN, n, statB):
            bn = st.bn
            return struct.pack("<qqddd12q", 1, statB, float(n), eps, bnm, P(bn.weight), P(bn.bias), 0, 0, 0, 0, 0, 0,
                               self._gptr(bn.weight), self._gptr(bn.bias), P(st.c1), P(st.c2))

        def tail(T, Cout, fins) -> int:
            if not use_tail:
                return 0
            # level-1 group size: <= 32 groups, so level 2 reads at most 32 fp64 group rows (bn_tail.h).  (Fewer,
            # larger level-1 groups - ~sqrt(2T) - measured 3.83-3.85 vs 3.78-3.79 ms/step at B=1024,
            # profiles/r3/resnet_epi_tail_ab.txt.)
            gs = max(8, -(-T // 32))
            NG = (T + gs - 1) // gs
            cnt = torch.zeros((Cout // 64) * (NG + 1), dtype=torch.int32, device=dev)
            self._keep.append(cnt)
            gpart = self._t((Cout // 64) * NG * 3 * 64, dtype=torch.float64)
            blob = struct.pack("<qqqq", cnt.data_ptr(), gpart.data_ptr(), gs, len(fins)) + b"".join(fins)
            blob += b"\0" * (304 - len(blob))
            tail_blobs.append(blob)
            if len(tail_blobs) > 160:
                raise RuntimeError("too many fused BatchNorm finalizes")
            return tails_dev.data_ptr() + 304 * (len(tail_blobs) - 1)

        # data-grad epilogues re-derive the BN1 ReLU mask from z1 and BN1's scale/shift instead of reading the stored
        # activation a1 (bitwise the same mask: the BN_ACT expression repeated; one activation read less per block).
        # BN-backward apply: one 8-channel vector per thread (several rows per thread at a fixed channel group -
        # per-channel coefficients loaded once - measured slower: 3.83-3.87 vs 3.79-3.80 ms/step at B=1024,
        # profiles/r2/resnet_multi_tile/bn_apply_rpt_ab.txt; BN1 + ReLU folded into conv2's register-staged
        # operand load measured slower than the LDS-DMA loop + BN_ACT pass: 3.85 vs 3.755,
        # profiles/r2/resnet_multi_tile/bn_fold_ab.txt - both removed in round 4)
        def conv(x, Lin, Cin, w_ptr, y, Lout, Cout, K, s, p, dil=1, st=None, add=None, add_mask=None, bnb=None,
                 tail_ptr=0, lane=0, mbn=None, pa=None, mask_bits=False):
            # bnb = (mask, z, mean, rstd, zd, mean_d, rstd_d): BN-backward statistics fused into the epilogue;
            # mbn = (scale, shift): the mask is relu(z * scale + shift) > 0 (mask operand not read);
            # pa = (scale, shift, out): the operand is relu(x * scale + shift), also stored to out (pre-activation);
            # mask_bits: bnb's mask is the bit mask a BN_ACT pass wrote (flag bit 1 of the relu word)
            extra = [P(t) if isinstance(t, torch.Tensor) else int(t or 0) for t in (bnb or ())]
            extra += [0] * (7 - len(extra))
            m_words = [P(mbn[0]), P(mbn[1])] if mbn is not None else [0, 0]
            pa_words = [P(t) for t in pa] if pa is not None else []
            op("CONV_FWD", P(x), w_ptr, 0, P(y), P(st), P(add), P(add_mask), B, Lin, Cin, Lout, Cout, K, s, p, dil,
               2 if mask_bits else 0, *extra, tail_ptr, *m_words, *pa_words, lane=lane)

        # BatchNorm + ReLU of a block's first conv folded into the second conv's operand staging (ECG_RESNET_PREACT=1,
        # default, where that conv is a 128-column tap-shared conv): the tap kernel applies relu(z1 * scale + shift)
        # to its staged image of z1 and stores a1 for the weight gradient - no BN_ACT pass over the tensor.  Bitwise
        # the BN_ACT pass (the same fmaf + max + bf16 rounding).
        use_preact = os.environ.get("ECG_RESNET_PREACT", "1") != "0"
        self.pre_act = use_preact

        def pre_act_ok(L_, C_in, C_out):
            return use_preact and bool(self.lib.ecg_conv1d_nlc_pa_ok(B, L_, C_in, L_, C_out, 3, 1, 1, 1))

        def wgrad(dy, x, Lin, Cin, Lout, Cout, K, s, p, weight):
            S = wsplits(B * Lout, Cout, K, Cin, s, Lin, Lout)
            op("CONV_WGRAD", P(dy), P(x), P(ws_w), S, B, Lin, Cin, Lout, Cout, K, s, p, lane=1)
            op("REDUCE_WGRAD", P(ws_w), S, Cout, K, Cin, self._gptr(weight), lane=1)

        # =============================== forward
        if self.source is not None:
            X, Y, table = self.source
            op("GATHER", P(X), X.stride(0), P(Y), P(table), P(self.counter), table.shape[0], B, L, P(self.x), P(self.y))
            op("COUNTER_INC", P(self.counter))
        op("WEIGHT_PREP", P(tab), len(convs), wprep_blocks, P(self.flat), P(self.warena))
        sr = self.lib.ecg_plan_stem_rows()
        T0 = (B * Lz + sr - 1) // sr
        op("STEM_FWD", P(self.x), P(c0.weight), P(self.z0), P(stats), B, L, Lz, Ks, Ss, Ps,
           tail(T0, 64, [fin_fwd_words(bn0, B * Lz)]))
        if not use_tail:
            fin_fwd(bn0, T0, B * Lz)
        op("STEM_POOL", P(self.z0), P(bn0.scale), P(bn0.shift), P(self.h0), B, Lz, Lp, 64, P(self.pool_am))
        xin = self.h0
        # side lane (with fused finalizes): a block's downsample conv runs beside conv1 -> BN_ACT -> conv2, on BN
        # partials of its own; the BN_ACT that adds it joins the lanes
        ds_side = side and use_tail
        stats_d = self._t(2 * max_T * 512, dtype=torch.float32) if ds_side else stats
        rows = lambda Lin, Cin, Lout, Cout, K, s, p, dil=1: self.lib.ecg_conv1d_nlc_fwd_stat_rows(  # noqa: E731
            B, Lin, Cin, Lout, Cout, K, s, p, dil)  # rows of the epilogue's BN partials for that exact conv
        for (Li, Ci, Lo, Co, s), blk, a, (b1, b2, bd) in zip(shapes, blocks, acts, bns):
            Td, T = rows(Li, Ci, Lo, Co, 1, s, 0), rows(Li, Ci, Lo, Co, 3, s, 1)
            if bd is not None and ds_side:
                conv(xin, Li, Ci, self._wf[id(blk.downsample[0])], a["zd"], Lo, Co, 1, s, 0, st=stats_d,
                     tail_ptr=tail(Td, Co, [fin_fwd_words(bd, B * Lo)]), lane=1)
            conv(xin, Li, Ci, self._wf[id(blk.conv1)], a["z1"], Lo, Co, 3, s, 1, st=stats,
                 tail_ptr=tail(T, Co, [fin_fwd_words(b1, B * Lo)]))
            if not use_tail:
                fin_fwd(b1, T, B * Lo)
            pre = pre_act_ok(Lo, Co, Co)
            if not pre:
                op("BN_ACT", 0, P(a["z1"]), P(b1.scale), P(b1.shift), 0, 0, 0, P(a["a1"]), B * Lo, Co)
            T2 = rows(Lo, Co, Lo, Co, 3, 1, 1)
            conv(a["z1"] if pre else a["a1"], Lo, Co, self._wf[id(blk.conv2)], a["z2"], Lo, Co, 3, 1, 1, st=stats,
                 tail_ptr=tail(T2, Co, [fin_fwd_words(b2, B * Lo)]), pa=(b1.scale, b1.shift, a["a1"]) if pre else None)
            if not use_tail:
                fin_fwd(b2, T2, B * Lo)
            if bd is not None:
                if not ds_side:
                    conv(xin, Li, Ci, self._wf[id(blk.downsample[0])], a["zd"], Lo, Co, 1, s, 0, st=stats,
                         tail_ptr=tail(Td, Co, [fin_fwd_words(bd, B * Lo)]))
                if not use_tail:
                    fin_fwd(bd, Td, B * Lo)
                op("BN_ACT", 2, P(a["z2"]), P(b2.scale), P(b2.shift), P(a["zd"]), P(bd.scale), P(bd.shift),
                   P(a["out"]), B * Lo, Co, P(a["mb"]), lane=2)
            else:
                op("BN_ACT", 1, P(a["z2"]), P(b2.scale), P(b2.shift), P(xin), 0, 0, P(a["out"]), B * Lo, Co, P(a["mb"]))
            a["in"] = xin
            xin = a["out"]

        # =============================== head (loss + dlogits + dW/db)
        seg_begin = len(ops)
        # op-range marks for per-block (teacher-forced) numerics checks: tests/test_resnet_engine_gpu.py
        self._blocks, self._shapes, self._acts, self._bns, self._bn0 = blocks, shapes, acts, bns, bn0
        self._fwd_end = seg_begin
        self._bwd_marks: List[Tuple[int, int, int, torch.Tensor, torch.Tensor]] = []
        gbuf = self._t(B, ncls, dtype=torch.float32)
        fbuf = self._t(B, self.Cf, dtype=torch.float32)
        lbuf = self._t(B, dtype=torch.float32)
        gcur = gA
        op("HEAD", P(xin), P(m.fc.weight), P(m.fc.bias), P(self.y), P(gcur), P(gbuf), P(fbuf), P(lbuf), B, self.Lf,
           self.Cf, ncls, 0)
        op("HEAD_REDUCE", P(gbuf), P(fbuf), P(lbuf), P(ws), B, self.Cf, ncls, Gb)
        if self.space.offset_of(m.fc.bias) != self.space.offset_of(m.fc.weight) + ncls * self.Cf:
            raise RuntimeError("fc.weight / fc.bias not adjacent in the flat buffer")
        op("REDUCE_SUM", P(ws), Gb, ncls * self.Cf + ncls + 1, self._gptr(m.fc.weight), ncls * self.Cf + ncls,
           P(self.loss_acc))

        # =============================== backward through the blocks (segments per stage)
        stage_of = []
        for si, st in enumerate((m.layer1, m.layer2, m.layer3, m.layer4)):
            stage_of += [si] * len(st)
        # BN-backward fusion: every data-grad conv's epilogue stores the ReLU-masked gradient and emits the
        # statistics (sum dz, sum dz*xhat [, sum dz*xhat_ds]) of the BatchNorm that consumes it; only the last
        # block (whose gradient comes from the head) runs a separate reduce pass.
        stats_b = self._t(3 * max_T * 512, dtype=torch.float32)  # cross-block BN2 statistics (conv1 dgrad -> next)
        nxt = gB
        seg_hi = self.space.param_numel
        bn2_src = None  # (partials base, T) of the current block's BN2 statistics
        for bi in range(len(blocks) - 1, -1, -1):
            (Li, Ci, Lo, Co, s), blk, a, (b1, b2, bd) = shapes[bi], blocks[bi], acts[bi], bns[bi]
            R = B * Lo
            blk_begin = len(ops)
            if side and bi < len(blocks) - 1:  # per-block BN-backward outputs (read by the side-stream wgrads)
                dz2, dz1, dzd = self._t(maxel), self._t(maxel), (self._t(maxel) if bd is not None else dzd)
            dzm, din = gcur, nxt  # dzm: ReLU-masked grad wrt this block's output
            if bn2_src is None:  # last block: gradient from the head
                ch = chunk_for(Co)
                Tb = (R + ch - 1) // ch
                fins = [fin_bwd_words(b2, R, 1)] + ([fin_bwd_words(bd, R, 2)] if bd is not None else [])
                op("BN_BWD_REDUCE", 3 if bd is not None else 2, P(gcur), P(a["out"]), P(a["z2"]), P(b2.mean),
                   P(b2.rstd), P(a.get("zd")), P(bd.mean) if bd else 0, P(bd.rstd) if bd else 0, P(bpart), R, Co, ch,
                   P(dzm), tail(Tb, Co, fins))
                bn2_src = (bpart.data_ptr(), Tb, use_tail)
            base, T2, fused = bn2_src
            if not fused:  # (fused: the data-grad conv that produced the statistics already finalized them)
                fin_bwd(b2, T2, R, 1, base)
                if bd is not None:
                    fin_bwd(bd, T2, R, 2, base)
            op("BN_BWD_APPLY", 1 if bd is not None else 0, P(dzm), 0, P(a["z2"]), P(b2.mean), P(b2.rstd),
               P(b2.scale), P(b2.c1), P(b2.c2), P(dz2), P(a.get("zd")), P(bd.mean) if bd else 0,
               P(bd.rstd) if bd else 0, P(bd.scale) if bd else 0, P(bd.c2) if bd else 0, P(dzd), R, Co)
            wgrad(dz2, a["a1"], Lo, Co, Lo, Co, 3, 1, 1, blk.conv2.weight)
            # dgrad conv2 (stride 1, pad 1) -> ReLU-masked grad wrt a1 + BN1 backward statistics
            T1 = rows(Lo, Co, Lo, Co, 3, 1, 1)
            conv(dz2, Lo, Co, self._wb[id(blk.conv2)], ga1, Lo, Co, 3, 1, 1, st=stats,
                 bnb=(a["a1"], a["z1"], b1.mean, b1.rstd, 0, 0, 0), tail_ptr=tail(T1, Co, [fin_bwd_words(b1, R, 1)]),
                 mbn=(b1.scale, b1.shift))
            if not use_tail:
                fin_bwd(b1, T1, R, 1, stats.data_ptr())
            op("BN_BWD_APPLY", 0, P(ga1), 0, P(a["z1"]), P(b1.mean), P(b1.rstd), P(b1.scale), P(b1.c1),
               P(b1.c2), P(dz1), 0, 0, 0, 0, 0, 0, R, Co)
            wgrad(dz1, a["in"], Li, Ci, Lo, Co, 3, s, 1, blk.conv1.weight)
            add = dzm
            if bd is not None:
                wgrad(dzd, a["in"], Li, Ci, Lo, Co, 1, s, 0, blk.downsample[0].weight)
                conv(dzd, Lo, Co, self._wb[id(blk.downsample[0])], tmp, Li, Ci, 1, 1, 0, dil=s)
                add = tmp
            if bi > 0:  # din is the previous block's output gradient: mask it and emit that block's BN2 stats
                pa, (_, pb2, pbd) = acts[bi - 1], bns[bi - 1]
                Tn = rows(Lo, Co, Li, Ci, 3, 1, 1, s)  # phase-decomposed when s > 1
                fins = [fin_bwd_words(pb2, B * Li, 1)] + ([fin_bwd_words(pbd, B * Li, 2)] if pbd else [])
                conv(dz1, Lo, Co, self._wb[id(blk.conv1)], din, Li, Ci, 3, 1, 1, dil=s, add=add, st=stats_b,
                     bnb=(pa["mb"], pa["z2"], pb2.mean, pb2.rstd, pa.get("zd") if pbd else 0,
                          pbd.mean if pbd else 0, pbd.rstd if pbd else 0), tail_ptr=tail(Tn, Ci, fins),
                     mask_bits=True)
                bn2_src = (stats_b.data_ptr(), Tn, use_tail)
            else:  # into the stem: plain gradient wrt the pooled activations
                conv(dz1, Lo, Co, self._wb[id(blk.conv1)], din, Li, Ci, 3, 1, 1, dil=s, add=add)
            # (block bi's ops: [blk_begin, len(ops)); they read dzm (the last block: unmasked, masked in place by
            # BN_BWD_REDUCE) and write din (ReLU-masked for block bi-1; the stem's unmasked pooled gradient at bi=0)
            self._bwd_marks.append((bi, blk_begin, len(ops), dzm, din))
            gcur, nxt = din, dzm
            # close a grad segment: at a stage boundary (bucket_mb = 0), or once the open segment's gradients
            # reach the bucket size; layer1's blocks join the stem segment either way
            boundary = bi == 0 or stage_of[bi - 1] != stage_of[bi]
            if stage_of[bi] == 0:
                if boundary:
                    break
                continue
            lo = min(self.space.offset_of(p) for p in blocks[bi].parameters())
            if (boundary and self.bucket_bytes <= 0) or (self.bucket_bytes > 0 and 4 * (seg_hi - lo) >= self.bucket_bytes):
                self._segments.append((seg_begin, len(ops), lo, seg_hi))
                seg_begin, seg_hi = len(ops), lo

        # =============================== stem backward
        Tb0 = (B * Lz + stem_chunk_b - 1) // stem_chunk_b
        op("STEM_BWD_REDUCE", P(gcur), P(self.z0), P(bn0.scale), P(bn0.shift), P(bn0.mean), P(bn0.rstd), P(dz0),
           P(bpart), B, Lz, Lp, 64, stem_chunk_b, tail(Tb0, 64, [fin_bwd_words(bn0, B * Lz, 1)]), P(self.pool_am))
        if not use_tail:
            fin_bwd(bn0, Tb0, B * Lz, 1)
        op("STEM_WGRAD", P(dz0), P(self.z0), P(bn0.mean), P(bn0.rstd), P(bn0.scale), P(bn0.c1), P(bn0.c2),
           P(self.x), P(ws), B, L, Lz, Ks, Ss, Ps, stem_chunk)
        op("REDUCE_SUM", P(ws), stem_blocks, 64 * Ks, self._gptr(c0.weight), 64 * Ks, 0)
        self._segments.append((seg_begin, len(ops), 0, seg_hi))
        self._fb_end = len(ops)
        # =============================== optimizer
        op("SGD", P(self.flat), P(self.grad), P(self.mom), self.space.param_numel, _f(self.lr), _f(self.momentum),
           _f(self.wd), int(self.nesterov), lane=2)
        if tail_blobs:
            blob = torch.frombuffer(bytearray(b"".join(tail_blobs)), dtype=torch.uint8)
            tails_dev[:blob.numel()].copy_(blob)
        self.n_bn_tails = len(tail_blobs)
        self.ops = torch.tensor(ops, dtype=torch.int64)
        self.n_ops = len(ops)
        # grad segments must tile [0, param_numel) back to front
        hi = self.space.param_numel
        for (_, _, lo, h) in self._segments:
            assert h == hi, (self._segments, hi)
            hi = lo
        assert hi == 0

    # ------------------------------------------------------------------------------------------ execution
    def _ops_ptr(self, begin: int) -> int:
        return self.ops.data_ptr() + 8 * OP_WORDS * begin

    def _run(self, begin: int, end: int):
        bad = ctypes.c_int(-1)
        st = self.lib.ecg_plan_run(self._ops_ptr(begin), end - begin, ctypes.byref(bad), _lib.stream_ptr(self.dev))
        if st:
            raise _lib.NativeError(f"resnet plan op {begin + bad.value} (kind {int(self.ops[begin + bad.value, 0])}) "
                                   f"failed with status {st}")

    def _graph(self, key: str, begin: int, end: int) -> int:
        h = self._graphs.get(key)
        if h is None:
            hp = ctypes.c_void_p()
            bad = ctypes.c_int(-1)
            st = self.lib.ecg_plan_graph_create(ctypes.byref(hp), self._ops_ptr(begin), end - begin,
                                                ctypes.byref(bad))
            if st:
                raise _lib.NativeError(f"resnet plan graph capture failed (status {st}, op {begin + bad.value})")
            h = self._graphs[key] = hp.value
        return h

    def _exec(self, key: str, begin: int, end: int):
        # With the side lane the plan runs eagerly: measured on MI355X (ResNet1D-34 B=1024, scripts/
        # diag_resnet_side.py) the fork-join plan takes 3.94 ms/step enqueued directly but 8.05 as a replayed
        # hipGraph (one stream: 4.56 either way).
        if self.use_graph and not self.side_lane:
            st = self.lib.ecg_plan_graph_launch(self._graph(key, begin, end), _lib.stream_ptr(self.dev))
            _lib.check(st, "ecg_plan_graph_launch")
        else:
            self._run(begin, end)

    def set_batch(self, x: torch.Tensor, y: torch.Tensor) -> None:
        self.x.copy_(x.reshape(self.B, self.L), non_blocking=True)
        self.y.copy_(y.reshape(self.B), non_blocking=True)

    def _run_nojoin(self, begin: int, end: int):
        """Enqueue ops [begin, end) without joining the side lane at the end; returns the side stream (a torch
        ExternalStream) when the range put work on it, else None."""
        bad = ctypes.c_int(-1)
        side = ctypes.c_void_p()
        st = self.lib.ecg_plan_run_ex(self._ops_ptr(begin), end - begin, ctypes.byref(bad), _lib.stream_ptr(self.dev),
                                      0, ctypes.byref(side))
        if st:
            raise _lib.NativeError(f"resnet plan op {begin + bad.value} failed with status {st}")
        if not side.value:
            return None
        if getattr(self, "_side_ext", None) is None or self._side_ext.cuda_stream != side.value:
            self._side_ext = torch.cuda.ExternalStream(side.value, device=self.dev)
        return self._side_ext

    def run_segments(self, on_segment: Callable[[int, int, int, Optional[torch.cuda.Stream]], None]) -> None:
        """Forward, then the backward one gradient bucket (segment) at a time: ``on_segment(i, lo, hi, side)`` is
        called once segment i's ops are enqueued, with the flat range [lo, hi) whose gradients they complete.  With
        the side lane the weight-gradient ops of the segment may still be running on ``side``: the callback orders
        its consumer (the bucket's all-reduce) after BOTH the current stream and ``side`` - the main stream itself
        never waits, so the data-gradient chain runs on beside the weight gradients and the collectives.  Ends
        with the side lane joined into the current stream (before the optimizer)."""
        first = self._segments[0][0]
        eager = not (self.use_graph and not self.side_lane)
        self._exec("fwd", 0, first)
        for i, (b, e, lo, hi) in enumerate(self._segments):
            if eager:
                side = self._run_nojoin(b, e)
            else:
                self._exec(f"seg{i}", b, e)
                side = None
            on_segment(i, lo, hi, side)
        if eager and self.side_lane:
            _lib.check(self.lib.ecg_plan_join(_lib.stream_ptr(self.dev)), "ecg_plan_join")
        self._loss_steps += 1
        self._steps_since_sync += 1

    def forward_backward(self) -> None:
        """Forward + backward into the flat grad buffer (``grad_sync`` per segment if set)."""
        if self.grad_sync is None:
            self._exec("fb", 0, self._fb_end)
        else:
            first = self._segments[0][0]
            self._exec("fwd", 0, first)
            for i, (b, e, lo, hi) in enumerate(self._segments):
                self._exec(f"seg{i}", b, e)
                self.grad_sync(self.grad[lo:hi])
        self._loss_steps += 1
        self._steps_since_sync += 1

    def apply_update(self) -> None:
        """The SGD op alone (after ``forward_backward`` and any gradient all-reduce)."""
        self._exec("sgd", self._fb_end, self.n_ops)

    def step(self) -> None:
        if self.grad_sync is None:
            self._exec("step", 0, self.n_ops)
            self._loss_steps += 1
            self._steps_since_sync += 1
        else:
            self.forward_backward()
            self.apply_update()

    def reset_counter(self) -> None:
        self.counter.zero_()

    def sgd_range(self, lo: int, hi: int, stream=None) -> None:
        """SGD on the flat parameter range [lo, hi) only (the per-segment update of ``--overlap tail``), on the
        current stream or ``stream``."""
        key = (lo, hi)
        ops = self._range_ops.get(key)
        if ops is None:
            w = [OP["SGD"], self.flat.data_ptr() + 4 * lo, self.grad.data_ptr() + 4 * lo, self.mom.data_ptr() + 4 * lo,
                 hi - lo, _f(self.lr), _f(self.momentum), _f(self.wd), int(self.nesterov)]
            ops = self._range_ops[key] = torch.tensor([w + [0] * (OP_WORDS - len(w))], dtype=torch.int64)
        bad = ctypes.c_int(-1)
        sp = stream.cuda_stream if stream is not None else _lib.stream_ptr(self.dev)
        st = self.lib.ecg_plan_run(ops.data_ptr(), 1, ctypes.byref(bad), sp)
        _lib.check(st, "ecg_plan_run(sgd_range)")

    def avg_loss(self) -> float:
        return float(self.loss_acc.item()) / max(1, self._loss_steps)

    def reset_loss(self) -> None:
        self.loss_acc.zero_()
        self._loss_steps = 0

    def reset_momentum(self) -> None:
        self.mom.zero_()

    def sync_counters(self) -> None:
        """Bring ``num_batches_tracked`` of every BN up to date (kept off the per-step plan)."""
        if self._steps_since_sync:
            with torch.no_grad():
                for st in self._bn_states:
                    st.bn.num_batches_tracked += self._steps_since_sync
            self._steps_since_sync = 0

    def close(self) -> None:
        for h in self._graphs.values():
            self.lib.ecg_plan_graph_destroy(h)
        self._graphs.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
