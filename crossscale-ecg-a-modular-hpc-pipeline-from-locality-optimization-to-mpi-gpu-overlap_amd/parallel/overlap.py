"""FedAvg communication with MEASURED overlap: one comm stream per device, one timing definition per backend.

Reference: the FedAvg round (TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:186-216) times its host-staged
collectives with ``perf_counter`` around blocking calls (:188-190, :209-211), so ``comm_ms`` is always fully
exposed.  Here every collective is issued through ``FedAvgComm`` - the ONLY comm-timing path (bench.py, the
FedAvg driver, the ResNet tail step and the tests all use it) - and two numbers are kept per collective:

* ``comm_ms`` - the collective's OWN span: from the moment it could start (its input is final) to its
  completion, on every backend;
* ``comm_exposed_ms`` - the time the compute side actually stalled on it (whatever weight-independent work was
  enqueued between issue and wait - the next round's batch staging for ``tail``, a whole local round for
  ``delayed``, the remaining backward segments of the ResNet tail step - shows up as the difference).

How each backend realises those points (``FedAvgComm.kind``):

``stream`` (GPU tensors on RCCL): the collective is issued from the device's comm stream (``comm_stream``, high
  priority) after that stream waited for the compute stream; RCCL's internal stream is ordered after it and
  ``work.wait()`` under the comm stream makes the COMM stream (not the compute stream) wait for RCCL.  hipEvents:
  ``issue``/``done`` on the comm stream (span), ``before``/``after`` around the compute stream's
  ``wait_event(done)`` (stall).
``host`` (CPU tensors, gloo): ``issue`` = host clock at the call (the input is final: CPU ops are synchronous),
  ``done`` = the clock when the work's future completed (a done-callback run by the backend's thread - the
  completion time, not the time the consumer looked; it can trail completion by up to one GIL switch interval when
  the main thread is running Python), stall = host time blocked in ``wait``.
``host_staged`` (GPU tensors over a host-staging backend, i.e. gloo rehearsing several ranks on one GPU): gloo
  copies the tensor to the host after the compute stream's pending work, so ``issue`` first synchronises the
  compute stream (that wait is compute, not communication), then as ``host``; the host blocks inside the issuing
  call (the staging copy) and in ``wait`` while the GPU runs only what was enqueued before it, so the host stall
  (both blocks, for every host kind) is the exposure.

``comm_stream(device)`` is shared by every issuer on a device (FedAvgComm, the ResNet trainer's DDP buckets and
tail SGD), so an N>1 rank runs on four streams: compute (torch's current stream), the engine's low-priority side
lane, this comm stream, and RCCL's internal stream (profiles/r6/stream_queues.txt audits the queue mapping).
"""
from __future__ import annotations

import contextlib
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch

from .env import DistContext
from .fedavg import allreduce_mean_

_COMM_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def comm_stream(device: torch.device) -> "torch.cuda.Stream":
    """The device's communication stream (created once, high priority): every collective issuer on the device
    uses it, so the stream count of a rank stays at compute + side lane + comm + RCCL's."""
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    s = _COMM_STREAMS.get(idx)
    if s is None:
        s = _COMM_STREAMS[idx] = torch.cuda.Stream(device=idx, priority=-1)
    return s


class Mark:
    """A point in time on a device stream (hipEvent) or on the host clock."""

    __slots__ = ("ev", "t")

    def __init__(self, stream: Optional[torch.cuda.Stream] = None, gpu: bool = False, t: Optional[float] = None):
        if gpu:
            self.ev = torch.cuda.Event(enable_timing=True)
            self.ev.record(stream or torch.cuda.current_stream())
            self.t = None
        else:
            self.ev = None
            self.t = time.perf_counter() if t is None else t

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
    completed_at: Optional[list] = None  # host kinds: [perf_counter at the work's completion] (done-callback)


@dataclass
class CommRecord:
    """Timing of one round's communication (resolved after the events completed)."""
    spans: List[tuple] = field(default_factory=list)  # (issue, done) per collective
    stalls: List[tuple] = field(default_factory=list)  # (before, after) on the compute stream / host
    blocking: List[tuple] = field(default_factory=list)  # synchronous collectives (broadcast): comm == exposed

    @property
    def first_issue(self) -> Optional[Mark]:
        return self.spans[0][0] if self.spans else None

    def comm_ms(self) -> float:
        """Blocking collectives plus the union span of the issued ones (first issue -> last completion)."""
        ms = sum(a.ms_to(b) for a, b in self.blocking)
        done = [d for _, d in self.spans if d is not None]
        if self.spans and done:
            first = self.spans[0][0]
            ms += max(first.ms_to(d) for d in done)
        return ms

    def exposed_ms(self) -> float:
        return sum(a.ms_to(b) for a, b in self.blocking) + sum(a.ms_to(b) for a, b in self.stalls)


def _completion_box(work) -> Optional[list]:
    """A list that receives ``perf_counter()`` when ``work`` completes (its future's done-callback), or None."""
    get = getattr(work, "get_future", None)  # fedavg._DivAfter: completes after its chained divide
    if get is None:
        return None
    try:
        fut = get()
    except Exception:  # backend without futures
        return None
    box: list = []
    fut.add_done_callback(lambda _f: box.append(time.perf_counter()))
    return box


class FedAvgComm:
    """Flat-buffer FedAvg collectives with per-collective timing marks (module docstring: the three kinds).

    ``allreduce(t, ctx, async_op=True)`` is the collective (default: ``fedavg.allreduce_mean_``, RCCL AVG /
    gloo SUM + divide); tests inject recorders."""

    def __init__(self, ctx: DistContext, allreduce: Optional[Callable] = None):
        self.ctx = ctx
        self.allreduce = allreduce or allreduce_mean_
        dev = getattr(ctx, "device", None)
        self.gpu = dev is not None and dev.type == "cuda"
        self.stream = None
        if self.gpu and getattr(ctx, "backend", "none") == "nccl":
            self.kind = "stream"
        elif self.gpu:
            self.kind = "host_staged"
        else:
            self.kind = "host"
        if self.kind == "stream" and ctx.distributed:
            self.stream = comm_stream(dev)

    def mark(self, stream=None) -> Mark:
        """A point on ``stream`` (GPU: hipEvent, for callers timing their own device work) / the host clock."""
        return Mark(stream, self.gpu)

    def _point(self, stream=None) -> Mark:
        """A timing point of this backend's kind (device event for ``stream``, host clock otherwise)."""
        return Mark(stream, self.kind == "stream")

    def issue(self, t: torch.Tensor, rec: CommRecord) -> Pending:
        """Start an all-reduce(AVG) of ``t`` once the compute stream's pending writes to it are done."""
        if not self.ctx.distributed:
            m = self._point()
            return Pending(None, m, m, True)
        if self.kind == "stream":
            compute = torch.cuda.current_stream(self.ctx.device)
            self.stream.wait_stream(compute)
            with torch.cuda.stream(self.stream):
                issue = self._point(self.stream)
                work = self.allreduce(t, self.ctx, async_op=True)
                if work is not None:
                    work.wait()  # comm stream waits for RCCL
                done = self._point(self.stream)
            t.record_stream(self.stream)
            p = Pending(None, issue, done)
        else:
            if self.kind == "host_staged":
                torch.cuda.current_stream(self.ctx.device).synchronize()  # t final: compute, not communication
            issue = self._point()
            work = self.allreduce(t, self.ctx, async_op=True)
            # the call itself can block the host (gloo copies CUDA tensors to the host inside it): exposed time too
            rec.stalls.append((issue, self._point()))
            p = Pending(work, issue, None, completed_at=_completion_box(work))
        rec.spans.append((p.issue, p.done))
        return p

    def wait(self, pendings: List[Pending], rec: CommRecord) -> None:
        """Make the compute stream (GPU) / the host (CPU) wait for ``pendings``; record the stall."""
        todo = [p for p in pendings if not p.waited]
        if not todo:
            return
        before = self._point()
        if self.kind == "stream":
            compute = torch.cuda.current_stream(self.ctx.device)
            for p in todo:
                compute.wait_event(p.done.ev)
                p.waited = True
            after = self._point()
        else:
            for p in todo:
                if p.work is not None:
                    p.work.wait()  # host_staged: also orders the compute stream after gloo's copy back
                p.waited = True
            after = self._point()
            for p in todo:
                box = p.completed_at
                if box is not None and not box:  # the callback needs the GIL: give the backend thread a chance
                    for _ in range(200):
                        time.sleep(0)
                        if box:
                            break
                p.done = Mark(t=min(box[0], after.t)) if box else after
                for i, (iss, d) in enumerate(rec.spans):
                    if iss is p.issue and d is None:
                        rec.spans[i] = (iss, p.done)
        rec.stalls.append((before, after))

    def blocking(self, fn, rec: CommRecord) -> None:
        """A synchronous collective (``fn()``) timed as fully exposed communication."""
        a = self._point()
        fn()
        rec.blocking.append((a, self._point()))


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
