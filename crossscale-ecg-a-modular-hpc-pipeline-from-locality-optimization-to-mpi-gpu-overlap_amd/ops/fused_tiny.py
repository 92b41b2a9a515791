"""Fused TinyECG training / inference on gfx950 (Python side of csrc/kernels/tiny_ecg_step.hip).

Each workgroup computes one sample's forward+backward out of LDS.  ``FusedTinyTrainer`` runs a whole FedAvg
local round as two launches per step (gradient slab, then slab reduction + SGD), captured into one native hipGraph
and replayed with a single ``hipGraphLaunch`` per round.  (A one-launch step with an in-kernel reduction tree and a
persistent one-launch round were measured slower on MI355X and removed in round 5: profiles/r4/tiny_phase_diag.txt.)

Reference semantics per step: Module_3/TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:103-132
(train_step_G0/G1), batches as Module_3/shard_dataset.py:118-136, optimizer SGD(lr=1e-2, momentum=0.9).
Differences: bf16 MFMA operands with fp32 accumulation (AMP numerics without a GradScaler), the loss is
accumulated on the device and read once per round (the reference syncs + ``loss.item()`` every step).
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import torch

from . import _lib
from ..models.tiny_ecg import TinyECG, num_params
from ..data.dataset import DeviceIndexSampler


PRECISION = {"bf16": 0, "fp32": 1}


def prec_id(precision: str) -> int:
    if precision not in PRECISION:
        raise ValueError(f"precision must be one of {list(PRECISION)}, got {precision!r}")
    return PRECISION[precision]


def prefrag_default() -> bool:
    """Prepared fragments (PF) on by default (``prefrag=False`` builds the conv operands in LDS every step: both
    paths are bitwise identical, csrc/kernels/tiny_ecg_step.hip WP_* comment)."""
    return True


def new_wprep(device) -> torch.Tensor:
    """Device buffer for the prepared-fragment image (bf16 conv operands of the flat weights, MFMA lane order).
    Zero-initialised: the K-padding slots are never written by the SGD epilogue that keeps the image current."""
    return torch.zeros(_lib.kernels().ecg_tiny_wprep_bytes(), dtype=torch.uint8, device=device)


def _wprep_ptr(precision: str, prefrag: Optional[bool], device, wprep: Optional[torch.Tensor] = None):
    if precision != "bf16" or not (prefrag_default() if prefrag is None else prefrag):
        return None, None
    w = new_wprep(device) if wprep is None else wprep
    return w.data_ptr(), w


def gather_default() -> bool:
    """PF round graphs gather every step's windows and labels into a contiguous ping-pong buffer inside the
    previous step's reduce launch (on by default; the ``gather`` attribute of a trainer), so the step kernel stages row b without the
    dependent idx -> window load (csrc/kernels/tiny_ecg_step.hip GatherArgs).  Measured: step kernel 7.76 -> 7.52
    us and step period 12.35 -> 12.08 us under the kernel tracer (medians of 687 steps), bench K=500 11.17 -> 11.06
    us/step (profiles/r3/tiny_gather_ab.txt)."""
    return True


def slab_stride(num_classes: int) -> int:
    return (num_params(num_classes) + 1 + 63) // 64 * 64


def _check_dataset(x: torch.Tensor, y: Optional[torch.Tensor], num_classes: int):
    if x.dim() != 2 or x.dtype != torch.float32 or not x.is_cuda or x.stride(1) != 1:
        raise ValueError(f"dataset must be a CUDA float32 [N, L] tensor with unit stride, got "
                         f"{x.dtype} {tuple(x.shape)} stride {x.stride()} on {x.device}")
    if y is not None:
        if y.dtype != torch.int32 or y.dim() != 1 or y.shape[0] != x.shape[0] or y.device != x.device:
            raise ValueError("labels must be int32 [N] on the dataset's device")


def _check_idx(idx: torch.Tensor, B: int, N: int, device):
    if idx.dtype != torch.int32 or idx.numel() < B or idx.device != device or not idx.is_contiguous():
        raise ValueError("idx must be a contiguous int32 device tensor with >= B entries")


def labels_int32(y: torch.Tensor, num_classes: int) -> torch.Tensor:
    y32 = y.to(torch.int32).contiguous()
    if y32.numel():
        lo, hi = int(y32.min()), int(y32.max())
        if lo < 0 or hi >= num_classes:
            raise ValueError(f"labels must be in [0, {num_classes}), got [{lo}, {hi}]")
    return y32


def tiny_forward(flat_params: torch.Tensor, x: torch.Tensor, idx: Optional[torch.Tensor], batch: int,
                 num_classes: int = 2, precision: str = "bf16", prefrag: Optional[bool] = None) -> torch.Tensor:
    """Logits [batch, C] of TinyECG for windows ``x[idx[b]]`` (or ``x[b]`` when idx is None).  ``prefrag``: build
    the prepared-fragment image first and run the PF kernel (default: ``prefrag_default()``)."""
    _check_dataset(x, None, num_classes)
    if idx is not None:
        _check_idx(idx, batch, x.shape[0], x.device)
    elif batch > x.shape[0]:
        raise ValueError("batch larger than dataset")
    out = torch.empty((batch, num_classes), dtype=torch.float32, device=x.device)
    lib = _lib.kernels()
    wp, _keep = _wprep_ptr(precision, prefrag, x.device)
    st = lib.ecg_tiny_forward(x.data_ptr(), x.shape[1], x.stride(0), _lib.ptr(idx), flat_params.data_ptr(),
                              num_classes, out.data_ptr(), batch, prec_id(precision), wp, _lib.stream_ptr(x.device))
    _lib.check(st, "ecg_tiny_forward")
    return out


def tiny_step_grads(flat_params: torch.Tensor, x: torch.Tensor, y32: torch.Tensor, idx: Optional[torch.Tensor],
                    batch: int, num_classes: int = 2, slab: Optional[torch.Tensor] = None,
                    precision: str = "bf16", prefrag: Optional[bool] = None,
                    wprep: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-sample gradient slab [batch, stride] (loss in column P) of one fused step (no update).  ``prefrag``:
    rebuild the prepared-fragment image (``wprep``, or a temporary) from the weights and run the PF kernel."""
    _check_dataset(x, y32, num_classes)
    if idx is not None:
        _check_idx(idx, batch, x.shape[0], x.device)
    stride = slab_stride(num_classes)
    if slab is None:
        slab = torch.empty((batch, stride), dtype=torch.float32, device=x.device)
    lib = _lib.kernels()
    wp, _keep = _wprep_ptr(precision, prefrag, x.device, wprep)
    st = lib.ecg_tiny_step_grads(x.data_ptr(), x.shape[1], x.stride(0), _lib.ptr(idx), y32.data_ptr(),
                                 flat_params.data_ptr(), num_classes, slab.data_ptr(), stride, batch,
                                 1.0 / batch, prec_id(precision), wp, _lib.stream_ptr(x.device))
    _lib.check(st, "ecg_tiny_step_grads")
    return slab


def reduce_slab(slab: torch.Tensor, num_classes: int = 2):
    """Sum a gradient slab: returns (grad [P], loss_sum [1]) without applying an update."""
    P = num_params(num_classes)
    grad = torch.empty(P, dtype=torch.float32, device=slab.device)
    loss = torch.zeros(1, dtype=torch.float32, device=slab.device)
    lib = _lib.kernels()
    st = lib.ecg_slab_reduce_sgd(slab.data_ptr(), slab.shape[0], slab.shape[1], P, None, None, grad.data_ptr(),
                                 loss.data_ptr(), 0.0, 0.0, 0.0, 0, 0, None, _lib.stream_ptr(slab.device))
    _lib.check(st, "ecg_slab_reduce_sgd")
    return grad, loss


class FusedTinyTrainer:
    """Single-GPU local trainer for TinyECG on the fused HIP step (one FL client).

    ``model`` is flattened in place: its parameters become views of ``self.params`` so that
    ``state_dict()`` / FedAvg collectives operate on the very buffer the kernels update.
    """

    def __init__(self, model: TinyECG, x_gpu: torch.Tensor, y_gpu: torch.Tensor, batch_size: int,
                 steps_per_round: int, lr: float = 1e-2, momentum: float = 0.9, weight_decay: float = 0.0,
                 nesterov: bool = False, seed: Optional[int] = None, use_graph: Optional[bool] = None,
                 precision: str = "bf16", prefrag: Optional[bool] = None):
        self.device = x_gpu.device
        self.precision = precision
        self.prec = prec_id(precision)
        self.model = model
        self.nc = model.num_classes
        self.params = model.flat if model.flat is not None else model.flatten_parameters()
        if self.params.device != self.device:
            raise ValueError("model and dataset must be on the same device")
        self.P = num_params(self.nc)
        self.x = x_gpu.contiguous()
        self.y32 = labels_int32(y_gpu, self.nc)
        _check_dataset(self.x, self.y32, self.nc)
        self.B = int(batch_size)
        self.S = int(steps_per_round)
        self.lr, self.momentum, self.wd, self.nesterov = float(lr), float(momentum), float(weight_decay), bool(nesterov)
        self.stride = slab_stride(self.nc)
        self.mom = torch.zeros_like(self.params)
        self.slab = torch.empty((self.B, self.stride), dtype=torch.float32, device=self.device)
        self.loss_acc = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.idx_table = torch.zeros((self.S, self.B), dtype=torch.int32, device=self.device)
        # batches of the NEXT round are drawn into idx_stage while the current round computes; each round graph
        # starts with a device copy idx_stage -> idx_table (csrc capture_round)
        self.idx_stage = torch.zeros((self.S, self.B), dtype=torch.int32, device=self.device)
        self._staged: Optional[int] = None  # rows staged for the next round (None: nothing staged)
        self.sampler = DeviceIndexSampler(self.x.shape[0], self.B, self.device, seed=seed)
        # a round = one hipGraph replay, or (ECG_TINY_GRAPH=0) the same kernels enqueued from a C++ loop
        self.use_graph = (os.environ.get("ECG_TINY_GRAPH", "1") != "0") if use_graph is None else bool(use_graph)
        self._graphs = {}  # n_steps -> native hipGraphExec handle
        self.steps_done = 0
        lib = _lib.kernels()
        smem = lib.ecg_tiny_smem_bytes(self.x.shape[1], self.prec)
        if smem > 160 * 1024:
            raise ValueError(f"window length {self.x.shape[1]} too long for the fused kernel ({smem} B LDS)")
        # prepared fragments (two-launch bf16 steps): a round's first step runs on the LDS path (the weights may
        # have been rewritten since: FedAvg, broadcast, checkpoint) and its SGD epilogue rewrites the whole image;
        # every later step of the round reads it
        pf = prefrag_default() if prefrag is None else bool(prefrag)
        self.prefrag = pf and precision == "bf16"
        self.wprep = new_wprep(self.device) if self.prefrag else None
        self.gather = gather_default() if self.prefrag else False
        self.xg = self.yg = None
        if self.gather:
            self.xg = torch.zeros(lib.ecg_tiny_gather_floats(self.x.shape[1], self.B), dtype=torch.float32,
                                  device=self.device)
            self.yg = torch.zeros(2 * self.B, dtype=torch.int32, device=self.device)

    # ------------------------------------------------------------------ graph management
    def _graph_for(self, n: int) -> C.c_void_p:
        # PF rounds read the staged table in place (no copy node) and the two index buffers swap roles after every
        # launch, so there is one graph per (size, buffer)
        key = (n, self.idx_stage.data_ptr()) if self.prefrag else n
        g = self._graphs.get(key)
        if g is not None:
            return g
        g = C.c_void_p()
        lib = _lib.kernels()
        torch.cuda.synchronize(self.device)
        if self.prefrag and self.gather:
            return self._part_graph(n, 0, key)
        else:
            tab, stage = (self.idx_stage, None) if self.prefrag else (self.idx_table, self.idx_stage)
            st = lib.ecg_round_graph_create(C.byref(g), self.x.data_ptr(), self.x.shape[1], self.x.stride(0),
                                            tab.data_ptr(), self.y32.data_ptr(), self.params.data_ptr(),
                                            self.mom.data_ptr(), self.nc, self.slab.data_ptr(), self.stride, self.B,
                                            n, self.loss_acc.data_ptr(), self.lr, self.momentum, self.wd,
                                            int(self.nesterov), self.prec,
                                            _lib.ptr(stage), _lib.ptr(self.wprep))
        _lib.check(st, "ecg_round_graph_create")
        self._graphs[key] = g
        return g

    def _part_graph(self, n: int, offset: int, key=None) -> C.c_void_p:
        """Graph of steps [offset, offset + n) of a PF round (offset 0: it runs the image-rebuilding first step),
        with the next-step gather when ``self.gather``."""
        key = key or ("part", n, offset, self.idx_stage.data_ptr())
        g = self._graphs.get(key)
        if g is not None:
            return g
        g = C.c_void_p()
        torch.cuda.synchronize(self.device)
        st = _lib.kernels().ecg_round_graph_create_pf(
            C.byref(g), self.x.data_ptr(), self.x.shape[1], self.x.stride(0), self.idx_stage.data_ptr(),
            self.y32.data_ptr(), self.params.data_ptr(), self.mom.data_ptr(), self.nc, self.slab.data_ptr(), self.stride,
            self.B, n, self.loss_acc.data_ptr(), self.lr, self.momentum, self.wd, int(self.nesterov),
            self.wprep.data_ptr(), offset, int(offset > 0), _lib.ptr(self.xg), _lib.ptr(self.yg))
        _lib.check(st, "ecg_round_graph_create_pf")
        self._graphs[key] = g
        return g

    def _round_graphs(self, n: int):
        """The graphs one replay of an n-step round launches, in order (one graph: a round split into a short head
        graph + the tail graph, so the GPU starts while the runtime still submits the tail, measured slower at
        every split - K=20: 11.8-12.0 vs 12.0-12.2 us/step, K=500: 10.89 vs 11.20, profiles/r3/
        tiny_head_split_ab.txt - and was removed)."""
        return [self._graph_for(n)]

    def _swap_tables(self) -> None:
        """After a PF graph launch: the buffer it read becomes ``idx_table`` (the last round's batches), the other
        one receives the next staging (enqueued behind the replay on the same stream)."""
        self.idx_table, self.idx_stage = self.idx_stage, self.idx_table

    def close(self):
        graphs, self._graphs = getattr(self, "_graphs", {}), {}
        for g in graphs.values():
            if g.value:
                _lib.kernels().ecg_round_graph_destroy(g)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ execution
    def _eager_step(self, s: int):
        lib = _lib.kernels()
        if self.prefrag:
            st = lib.ecg_tiny_train_step_pf(self.x.data_ptr(), self.x.shape[1], self.x.stride(0),
                                            self.idx_table[s].data_ptr(), self.y32.data_ptr(), self.params.data_ptr(),
                                            self.mom.data_ptr(), self.nc, self.slab.data_ptr(), self.stride, self.B,
                                            self.loss_acc.data_ptr(), self.lr, self.momentum, self.wd,
                                            int(self.nesterov), self.wprep.data_ptr(), int(s > 0),
                                            _lib.stream_ptr(self.device))
            _lib.check(st, "ecg_tiny_train_step_pf")
            return
        st = lib.ecg_tiny_train_step(self.x.data_ptr(), self.x.shape[1], self.x.stride(0),
                                     self.idx_table[s].data_ptr(), self.y32.data_ptr(), self.params.data_ptr(),
                                     self.mom.data_ptr(), self.nc, self.slab.data_ptr(), self.stride, self.B,
                                     self.loss_acc.data_ptr(), self.lr, self.momentum, self.wd, int(self.nesterov),
                                     self.prec, _lib.ptr(self.wprep),
                                     _lib.stream_ptr(self.device))
        _lib.check(st, "ecg_tiny_train_step")

    def prepare(self, sizes) -> None:
        """Draw the sampler's first permutation block, then capture, upload and warm every round graph whose step
        count is in ``sizes``, so a later round of that size only replays.  The warm-up replay is rolled back (weights, momentum, loss, staged batches are
        restored): it leaves the training state exactly as it found it."""
        self.sampler.prime()
        if not self.use_graph:
            return
        lib = _lib.kernels()
        sizes = [self._check_n(n) for n in sizes]
        state = (self.params, self.mom, self.loss_acc, self.idx_stage, self.idx_table)
        snap = [t.clone() for t in state]
        stream = _lib.stream_ptr(self.device)
        for n in sizes:
            for _ in range(2 if self.prefrag else 1):  # PF: both index buffers
                for g in self._round_graphs(n):
                    _lib.check(lib.ecg_round_graph_upload(g, stream), "ecg_round_graph_upload")
                    _lib.check(lib.ecg_round_graph_launch(g, stream), "ecg_round_graph_launch")
                if self.prefrag:
                    self._swap_tables()
        for t, v in zip(state, snap):
            t.copy_(v)
        torch.cuda.synchronize(self.device)

    def _check_n(self, n_steps: Optional[int]) -> int:
        n = self.S if n_steps is None else int(n_steps)
        if not 0 < n <= self.S:
            raise ValueError(f"n_steps must be in [1, {self.S}]")
        return n

    def stage(self, n_steps: Optional[int] = None) -> None:
        """Draw the next round's ``n_steps`` batches into the staging table (enqueued on the current stream: it
        runs after the rounds already enqueued, which read the staging table at their start)."""
        n = self._check_n(n_steps)
        self.sampler.fill(self.idx_stage[:n])
        self._staged = n

    def prepare_round(self, n_steps: Optional[int] = None, reset_loss: bool = True) -> None:
        """Batch preparation of a round (unless ``launch_round(..., next_n=n)`` already staged it); reads no
        weights, so it can run while the previous round's FedAvg all-reduce is in flight (``--overlap tail``)."""
        n = self._check_n(n_steps)
        if reset_loss:
            self.loss_acc.zero_()
            self._loss_steps = 0
        if self._staged != n:
            if self._staged is not None:
                raise RuntimeError(f"{self._staged} rows are staged for the next round, not {n}")
            self.stage(n)

    def run_round(self, n_steps: Optional[int] = None, reset_loss: bool = True, next_n: Optional[int] = None) -> None:
        """Enqueue ``n_steps`` (default ``steps_per_round``) local SGD steps on the current stream (async);
        ``next_n``: also stage the following round's batches behind this round."""
        self.prepare_round(n_steps, reset_loss)
        self.launch_round(n_steps, next_n)

    def launch_round(self, n_steps: Optional[int] = None, next_n: Optional[int] = None) -> None:
        """The round's SGD steps on the staged batches (one graph replay), then optionally stage the next round."""
        n = self._check_n(n_steps)
        if self._staged != n:
            raise RuntimeError("launch_round without prepare_round: no batches staged for this round")
        self._staged = None
        if self.use_graph:
            stream = _lib.stream_ptr(self.device)
            for g in self._round_graphs(n):
                _lib.check(_lib.kernels().ecg_round_graph_launch(g, stream), "ecg_round_graph_launch")
            if self.prefrag:
                self._swap_tables()
        elif self.prefrag:  # the graph's kernels enqueued from one C++ loop, reading the staged table in place
            _lib.check(_lib.kernels().ecg_tiny_train_steps_pf(
                self.x.data_ptr(), self.x.shape[1], self.x.stride(0), self.idx_stage.data_ptr(), self.y32.data_ptr(),
                self.params.data_ptr(), self.mom.data_ptr(), self.nc, self.slab.data_ptr(), self.stride, self.B, n,
                self.loss_acc.data_ptr(), self.lr, self.momentum, self.wd, int(self.nesterov),
                self.wprep.data_ptr(), 0, _lib.stream_ptr(self.device)), "ecg_tiny_train_steps_pf")
            self._swap_tables()
        else:
            self.idx_table[:n].copy_(self.idx_stage[:n])
            for s in range(n):
                self._eager_step(s)
        self.steps_done += n
        self._loss_steps = getattr(self, "_loss_steps", 0) + n
        if next_n is not None:
            self.stage(next_n)

    def avg_loss(self) -> float:
        """Mean per-step loss since the last reset (synchronises)."""
        return float(self.loss_acc.item()) / (self.B * max(1, getattr(self, "_loss_steps", self.S)))

    def reset_momentum(self):
        self.mom.zero_()
