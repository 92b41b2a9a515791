"""FedAvg communication with MEASURED overlap: a dedicated comm stream, hipEvents on both streams.

Reference: the FedAvg round (TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:186-216) times its host-staged
collectives with ``perf_counter`` around blocking calls (:188-190, :209-211), so ``comm_ms`` is always fully
exposed.  Here every collective is issued from a high-priority comm stream that first waits on an event of
the compute stream; RCCL's internal stream is ordered after the comm stream, and ``work.wait()`` issued under
the comm stream makes the COMM stream (not the compute stream) wait for RCCL.  Four events per collective:

* ``issue``  (comm stream, after it waited for the weights to be final) and ``done`` (comm stream, after RCCL
  finished): ``comm_ms = issue -> done`` is the collective's own duration;
* ``before`` and ``after`` (compute stream) around the compute stream's wait on ``done``:
  ``exposed_ms = before -> after`` is the time the compute stream actually stalled on communication.

So ``comm_exposed_ms`` is measured, not copied from ``comm_ms``: whatever compute stream work was enqueued
between issue and wait (next round's batch preparation for ``tail``, a whole local round for ``delayed``, the
earlier backward segments of the ResNet tail step) shows up as the difference.

On CPU (gloo) the same API uses host clocks: ``comm_ms`` = issue -> completion observed by ``wait`` and
``exposed_ms`` = time blocked inside ``wait``.
"""
from __future__ import annotations

import contextlib
import time
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from .env import DistContext
from .fedavg import allreduce_mean_


class Mark:
    """A point in time on a device stream (hipEvent) or on the host clock."""

    __slots__ = ("ev", "t")

    def __init__(self, stream: Optional[torch.cuda.Stream] = None, gpu: bool = False):
        if gpu:
            self.ev = torch.cuda.Event(enable_timing=True)
            self.ev.record(stream or torch.cuda.current_stream())
            self.t = None
        else:
            self.ev = None
            self.t = time.perf_counter()

    def ms_to(self, other: "Mark") -> float:
        if self.ev is not None:
            other.ev.synchronize()
            return float(self.ev.elapsed_time(other.ev))
        return (other.t - self.t) * 1e3


@dataclass
class Pending:
    """One in-flight collective."""
    work: object = None
    issue: Optional[Mark] = None
    done: Optional[Mark] = None
    waited: bool = False


@dataclass
class CommRecord:
    """Timing of one round's communication (resolved after the events completed)."""
    first_issue: Optional[Mark] = None
    last_done: Optional[Mark] = None
    stalls: List[tuple] = field(default_factory=list)  # (before, after) on the compute stream
    blocking: List[tuple] = field(default_factory=list)  # synchronous collectives (broadcast): comm == exposed

    def comm_ms(self) -> float:
        ms = sum(a.ms_to(b) for a, b in self.blocking)
        if self.first_issue is not None and self.last_done is not None:
            ms += self.first_issue.ms_to(self.last_done)
        return ms

    def exposed_ms(self) -> float:
        return sum(a.ms_to(b) for a, b in self.blocking) + sum(a.ms_to(b) for a, b in self.stalls)


class FedAvgComm:
    """Flat-buffer FedAvg collectives on a dedicated comm stream with per-collective timing marks."""

    def __init__(self, ctx: DistContext):
        self.ctx = ctx
        self.gpu = ctx.device.type == "cuda"
        self.stream = None
        if self.gpu and ctx.distributed:
            self.stream = torch.cuda.Stream(device=ctx.device, priority=-1)

    def mark(self, stream=None) -> Mark:
        return Mark(stream, self.gpu)

    def issue(self, t: torch.Tensor, rec: CommRecord) -> Pending:
        """Start an all-reduce(AVG) of ``t`` once the compute stream's pending writes to it are done."""
        if not self.ctx.distributed:
            m = self.mark()
            if rec.first_issue is None:
                rec.first_issue = m
            rec.last_done = m
            return Pending(None, m, m, True)
        if self.gpu:
            compute = torch.cuda.current_stream(self.ctx.device)
            self.stream.wait_stream(compute)
            with torch.cuda.stream(self.stream):
                issue = self.mark(self.stream)
                work = allreduce_mean_(t, self.ctx, async_op=True)
                if work is not None:
                    work.wait()  # comm stream waits for RCCL (and runs gloo's divide, if any)
                done = self.mark(self.stream)
            t.record_stream(self.stream)
            p = Pending(None, issue, done)
        else:
            issue = self.mark()
            p = Pending(allreduce_mean_(t, self.ctx, async_op=True), issue)
        if rec.first_issue is None:
            rec.first_issue = p.issue
        return p

    def wait(self, pendings: List[Pending], rec: CommRecord) -> None:
        """Make the compute stream (GPU) / the host (CPU) wait for ``pendings``; record the stall."""
        todo = [p for p in pendings if not p.waited]
        if not todo:
            return
        before = self.mark()
        if self.gpu:
            compute = torch.cuda.current_stream(self.ctx.device)
            for p in todo:
                compute.wait_event(p.done.ev)
                p.waited = True
            after = self.mark()
        else:
            for p in todo:
                if p.work is not None:
                    p.work.wait()
                p.waited = True
            after = self.mark()
            for p in todo:
                p.done = after
        rec.stalls.append((before, after))
        rec.last_done = todo[-1].done

    def blocking(self, fn, rec: CommRecord) -> None:
        """A synchronous collective (``fn()``) timed as fully exposed communication."""
        a = self.mark()
        fn()
        rec.blocking.append((a, self.mark()))


class FedAvgRound:
    """FedAvg round ending for one client, in one of the overlap modes.

    * ``none``: all-reduce(AVG) of the final weights; the compute stream waits right away (exact FedAvg);
    * ``tail``: the same collective, but the compute stream first enqueues the NEXT round's batch preparation
      (``before_wait``) and only then waits - exact FedAvg, bitwise equal to ``none``;
    * ``delayed``: one-round-stale FedAvg - the all-reduce of a snapshot of round r's weights runs under round
      r+1's local steps; at the next boundary ``w <- w + (avg_r - w_r)`` (changes the algorithm, opt-in).

    ``end_round(rec)`` is called after the round's local steps are enqueued; ``begin_round(rec_prev, prep)``
    before the next round's steps: it runs ``prep`` (weight-independent work) and then waits.
    """

    def __init__(self, flat: torch.Tensor, comm: FedAvgComm, mode: str = "none"):
        if mode not in ("none", "tail", "delayed"):
            raise ValueError(f"unknown overlap mode {mode!r}")
        self.flat, self.comm, self.mode = flat, comm, mode
        self._pending: List[Pending] = []
        self._rec: Optional[CommRecord] = None
        if mode == "delayed":
            self.snap = torch.empty_like(flat)
            self.base = torch.empty_like(flat)

    @property
    def in_flight(self) -> bool:
        return bool(self._pending)

    def end_round(self, rec: CommRecord) -> None:
        if self.mode == "delayed":
            self._finish_delayed()
            self.base.copy_(self.flat)
            self.snap.copy_(self.flat)
            self._pending = [self.comm.issue(self.snap, rec)]
            self._rec = rec
            return
        p = self.comm.issue(self.flat, rec)
        if self.mode == "none":
            self.comm.wait([p], rec)
        else:
            self._pending, self._rec = [p], rec

    def begin_round(self, prep=None) -> None:
        """Weight-independent work for the next round, then (tail) the wait for the averaged weights."""
        if prep is not None:
            prep()
        if self.mode == "tail" and self._pending:
            self.comm.wait(self._pending, self._rec)
            self._pending, self._rec = [], None

    def _finish_delayed(self) -> None:
        if not self._pending:
            return
        self.comm.wait(self._pending, self._rec)
        self._pending, self._rec = [], None
        self.flat.add_(self.snap).sub_(self.base)  # w <- w + (avg_r - w_r)

    @contextlib.contextmanager
    def averaged_in_place(self):
        """Inside the block ``flat`` holds the last all-reduced average (``delayed``: avg_r, after a stream wait on
        the in-flight collective, which stays pending - the stale correction is still applied at the next
        boundary); on exit ``flat`` is restored.  Other modes: ``flat`` is already the average, nothing changes."""
        if self.mode != "delayed" or not self._pending:
            yield
            return
        self.comm.wait(self._pending, self._rec)  # marks them waited; _finish_delayed later only applies
        keep = self.flat.clone()
        with torch.no_grad():
            self.flat.copy_(self.snap)
        try:
            yield
        finally:
            with torch.no_grad():
                self.flat.copy_(keep)

    def finalize(self) -> None:
        """Drain an in-flight collective (end of training)."""
        if self.mode == "delayed":
            self._finish_delayed()
        elif self._pending:
            self.comm.wait(self._pending, self._rec)
            self._pending, self._rec = [], None
