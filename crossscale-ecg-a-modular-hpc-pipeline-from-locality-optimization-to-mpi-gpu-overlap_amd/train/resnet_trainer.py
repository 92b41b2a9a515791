"""ResNet1D client trainer on the native step engine (ops.resnet_engine) - BASELINE.json config 5.

Same interface as ``TorchLocalTrainer`` / ``FusedTinyTrainer`` (``run_round`` / ``avg_loss`` /
``reset_momentum`` / ``close`` / ``mom``) so ``train.fedavg.run_fedavg`` drives it unchanged:

* per round: one ``randperm`` fill of the [S, B] index table, a counter reset, then S replays of the captured
  step graph (batch gather -> forward -> backward -> SGD, all on device; no host work per step);
* ``sync="ddp"``: synchronous data parallel - each backward segment's gradient range is all-reduced (RCCL AVG,
  async) as soon as the segment's graph is enqueued, so the reduction of layer4's gradients overlaps the
  backward of layer3..stem; the SGD op waits on the collectives on the GPU (no host sync);
* ``tail_fedavg()``: the ``--overlap tail`` round ending (SURVEY §5.8 mode 2) - the last step's SGD is applied
  per segment and each segment's updated weights are all-reduced while earlier segments still run backward;
  the result equals ``none`` FedAvg (all-reduce of the final weights) up to fp32 summation order.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from ..data.dataset import DeviceIndexSampler
from ..ops.resnet_engine import ResNetStepEngine
from ..parallel.env import DistContext
from ..parallel.fedavg import allreduce_mean_


class ResNetEngineTrainer:
    def __init__(self, model, x: torch.Tensor, y: torch.Tensor, batch_size: int, steps_per_round: int,
                 lr: float = 1e-2, momentum: float = 0.9, weight_decay: float = 0.0, seed: Optional[int] = None,
                 use_graph: bool = True, ctx: Optional[DistContext] = None, sync: str = "fedavg"):
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
                                       grad_sync=self._grad_sync if ddp else None,
                                       source=(self.x, self.y32, self.table))
        self.mom = self.engine.mom
        self.steps_done = 0

    def _grad_sync(self, seg: torch.Tensor) -> None:
        self._works.append(allreduce_mean_(seg, self.ctx, async_op=True))

    def _wait(self) -> None:
        for w in self._works:
            if w is not None:
                w.wait()
        self._works.clear()

    def _step(self) -> None:
        if self.engine.grad_sync is None:
            self.engine.step()
        else:
            self.engine.forward_backward()
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
        """Run one more local step whose update is applied and all-reduced segment by segment (exact FedAvg of
        the post-step weights, communication overlapped with the remaining backward).

        ``comm``/``rec`` (``parallel.overlap.FedAvgComm`` / ``CommRecord``): issue the collectives from the
        timed comm stream so the round records the collectives' span and the compute stream's actual stall."""
        eng = self.engine
        if self.ctx is None or not self.ctx.distributed:
            self._step()
            return
        if comm is None:
            from ..parallel.overlap import CommRecord, FedAvgComm
            comm, rec = FedAvgComm(self.ctx), CommRecord()
        first = eng._segments[0][0]
        eng._exec("fwd", 0, first)
        pend = []
        for i, (b, e, lo, hi) in enumerate(eng._segments):
            eng._exec(f"seg{i}", b, e)
            eng.sgd_range(lo, hi)
            pend.append(comm.issue(eng.flat[lo:hi], rec))
        eng._loss_steps += 1
        eng._steps_since_sync += 1
        # BN running statistics (not touched by SGD) are averaged too, like the flat all-reduce of ``none``
        buf = eng.flat[eng.space.param_numel:]
        if buf.numel():
            pend.append(comm.issue(buf, rec))
        comm.wait(pend, rec)
        self.steps_done += 1

    def avg_loss(self) -> float:
        return self.engine.avg_loss()

    def reset_momentum(self) -> None:
        self.engine.reset_momentum()

    def close(self) -> None:
        self.engine.sync_counters()
        self.engine.close()
