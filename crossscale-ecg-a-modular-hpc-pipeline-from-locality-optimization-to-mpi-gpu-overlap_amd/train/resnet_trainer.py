"""ResNet1D client trainer on the native step engine (ops.resnet_engine) - BASELINE.json config 5.

Same interface as ``TorchLocalTrainer`` / ``FusedTinyTrainer`` (``run_round`` / ``avg_loss`` /
``reset_momentum`` / ``close`` / ``mom``) so ``train.fedavg.run_fedavg`` drives it unchanged:

* per round: one ``randperm`` fill of the [S, B] index table, a counter reset, then S replays of the captured
  step graph (batch gather -> forward -> backward -> SGD, all on device; no host work per step);
* ``sync="ddp"``: synchronous data parallel - the backward runs in gradient buckets of ~``bucket_mb`` (4 MB;
  ``ResNetStepEngine.run_segments``) and each bucket's gradient range is all-reduced (RCCL AVG, async) from a
  comm stream ordered after the bucket's ops on BOTH the main stream and the weight-gradient side lane - the
  main stream never waits, so layer4's first bucket reduces while the rest of the backward runs; the SGD op
  waits on the collectives on the GPU (no host sync);
* ``tail_fedavg()``: the ``--overlap tail`` round ending (SURVEY §5.8 mode 2) - the last step's SGD is applied
  per bucket (on the comm stream, after the bucket's gradients are final) and each bucket's updated weights are
  all-reduced while earlier buckets still run backward; the result equals ``none`` FedAvg (all-reduce of the
  final weights) up to fp32 summation order.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..data.dataset import DeviceIndexSampler
from ..ops.resnet_engine import ResNetStepEngine
from ..parallel.env import DistContext
from ..parallel.fedavg import allreduce_mean_
from ..parallel.overlap import comm_stream


class ResNetEngineTrainer:
    def __init__(self, model, x: torch.Tensor, y: torch.Tensor, batch_size: int, steps_per_round: int,
                 lr: float = 1e-2, momentum: float = 0.9, weight_decay: float = 0.0, seed: Optional[int] = None,
                 use_graph: bool = True, ctx: Optional[DistContext] = None, sync: str = "fedavg",
                 bucket_mb: Optional[float] = None):
        self.model, self.B, self.S = model, batch_size, steps_per_round
        self.ctx = ctx
        self.device = x.device
        self.x = x.contiguous()
        self.y32 = y.to(torch.int32).contiguous()
        self.table = torch.zeros((steps_per_round, batch_size), dtype=torch.int32, device=self.device)
        self.sampler = DeviceIndexSampler(x.shape[0], batch_size, self.device, seed=seed)
        self._works: List = []
        ddp = sync == "ddp" and ctx is not None and ctx.distributed
        self.engine = ResNetStepEngine(model, batch_size, x.shape[1], lr=lr, momentum=momentum,
                                       weight_decay=weight_decay, use_graph=use_graph,
                                       source=(self.x, self.y32, self.table), bucket_mb=bucket_mb)
        self.ddp = ddp
        # the device's one comm stream (shared with parallel.overlap.FedAvgComm: compute + side lane + comm + RCCL's)
        self._comm = comm_stream(self.device) if ctx is not None and ctx.distributed and self.device.type == "cuda" \
            else None
        self.issue_log: List = []  # (segment, lo, hi) in issue order (tests / timeline)
        self.mom = self.engine.mom
        self.steps_done = 0

    def _after(self, side) -> torch.cuda.Stream:
        """The comm stream, ordered after everything enqueued so far on the current stream and on ``side``."""
        self._comm.wait_stream(torch.cuda.current_stream(self.device))
        if side is not None:
            self._comm.wait_stream(side)
        return self._comm

    def _wait(self) -> None:
        for w in self._works:
            if w is not None:
                w.wait()  # the current (main) stream waits for the collective
        self._works.clear()
        torch.cuda.current_stream(self.device).wait_stream(self._comm)

    def _step(self) -> None:
        if not self.ddp:
            self.engine.step()
        else:
            def bucket(i, lo, hi, side):
                with torch.cuda.stream(self._after(side)):
                    self.issue_log.append((i, lo, hi))
                    self._works.append(allreduce_mean_(self.engine.grad[lo:hi], self.ctx, async_op=True))
            self.engine.run_segments(bucket)
            self._wait()  # stream-side wait on the RCCL collectives, then SGD
            self.engine.apply_update()
        self.steps_done += 1

    def stage(self, n: Optional[int] = None) -> None:
        """Draw the NEXT round's batches into the index table, enqueued behind the rounds already launched (which
        have consumed it); no weights read, so it runs beside an in-flight all-reduce."""
        # the whole round's batches are drawn up front (a round ended by ``tail_fedavg`` uses the last row)
        self.sampler.fill(self.table)
        self._staged = True

    def prepare_round(self, n: Optional[int] = None, reset_loss: bool = True) -> None:
        """Draw the round's batches into the index table unless ``stage`` already did."""
        n = self.S if n is None else n
        if n > self.S:
            raise ValueError(f"round of {n} steps > steps_per_round={self.S}")
        if reset_loss:
            self.engine.reset_loss()
        if not getattr(self, "_staged", False):
            self.sampler.fill(self.table)
        self._staged = False
        self.engine.reset_counter()

    def launch_round(self, n: Optional[int] = None, next_n: Optional[int] = None) -> None:
        n = self.S if n is None else n
        for _ in range(n):
            self._step()

    def run_round(self, n: Optional[int] = None, reset_loss: bool = True) -> None:
        self.prepare_round(n, reset_loss)
        self.launch_round(n)

    run_steps = run_round

    def tail_fedavg(self, comm=None, rec=None) -> None:
        """Run one more local step whose update is applied and all-reduced bucket by bucket (exact FedAvg of the
        post-step weights, communication overlapped with the remaining backward).

        ``comm``/``rec`` (``parallel.overlap.FedAvgComm`` / ``CommRecord``): issue the collectives from the
        timed comm stream so the round records the collectives' span and the compute stream's actual stall."""
        eng = self.engine
        if self.ctx is None or not self.ctx.distributed:
            self._step()
            return
        if comm is None:
            from ..parallel.overlap import CommRecord, FedAvgComm
            comm, rec = FedAvgComm(self.ctx), CommRecord()
        pend = []
        upd = self._comm if comm.stream is None else comm.stream

        def bucket(i, lo, hi, side):
            # the bucket's SGD runs on the comm stream once its gradients are final on both lanes; FedAvgComm.issue
            # orders the all-reduce after the current stream, so issue it from the comm stream itself
            upd.wait_stream(torch.cuda.current_stream(self.device))
            if side is not None:
                upd.wait_stream(side)
            with torch.cuda.stream(upd):
                eng.sgd_range(lo, hi, stream=upd)
                self.issue_log.append((i, lo, hi))
                pend.append(comm.issue(eng.flat[lo:hi], rec))

        eng.run_segments(bucket)
        # BN running statistics (not touched by SGD) are averaged too, like the flat all-reduce of ``none``
        buf = eng.flat[eng.space.param_numel:]
        if buf.numel():
            pend.append(comm.issue(buf, rec))
        comm.wait(pend, rec)
        torch.cuda.current_stream(self.device).wait_stream(upd)
        self.steps_done += 1

    def avg_loss(self) -> float:
        return self.engine.avg_loss()

    def reset_momentum(self) -> None:
        self.engine.reset_momentum()

    def close(self) -> None:
        self.engine.sync_counters()
        self.engine.close()
