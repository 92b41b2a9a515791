"""Timers: host wall clock with device fences, and hipEvent-based per-stream timers.

Reference timing is ``time.perf_counter()`` bracketed by ``torch.cuda.synchronize()``
(bench_locality.py:44-66, part3_fedavg...py:188-211).  ``WallTimer`` reproduces that exactly;
``StreamTimer`` measures work on one stream with hipEvents (no host sync inside the timed region) so
copy/compute/comm overlap can be measured rather than assumed.
"""
from __future__ import annotations

import time
from contextlib import contextmanager
from typing import Optional

import torch


def sync(device: Optional[torch.device]) -> None:
    if device is not None and torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def warm_until_stable(step, device=None, min_steps: int = 5, max_steps: int = 200, window: int = 5,
                      tol: float = 1.5) -> int:
    """Untimed warm-up: run ``step()`` (synchronised) at least ``min_steps`` times and until the last ``window``
    step times are all within ``tol`` x their minimum, at most ``max_steps``.  Returns the steps run.

    A fixed 5-step warm-up (the reference's, bench_locality.py:29-38) is not enough on a fresh MI355X box: MIOpen
    compiles some solvers' kernels at first use, and a compile that lands in the timed loop inflates the mean
    step time by its whole duration (round 1: A4 at B=256 and G1_overlap_amp read 3-20x slower)."""
    times = []
    for i in range(max_steps):
        t0 = time.perf_counter()
        step()
        sync(device)
        times.append(time.perf_counter() - t0)
        if i + 1 >= max(min_steps, window):
            last = times[-window:]
            if max(last) <= tol * min(last):
                return i + 1
    return max_steps


class WallTimer:
    def __init__(self, device=None):
        self.device = device
        self.ms = 0.0

    @contextmanager
    def __call__(self, fence: bool = True):
        if fence:
            sync(self.device)
        t0 = time.perf_counter()
        yield self
        if fence:
            sync(self.device)
        self.ms += (time.perf_counter() - t0) * 1e3


class StreamTimer:
    """Accumulates elapsed time of regions enqueued on a stream (read with ``elapsed_ms()``)."""

    def __init__(self, stream: Optional[torch.cuda.Stream] = None):
        self.stream = stream
        self.pairs = []

    @contextmanager
    def region(self):
        s = self.stream or torch.cuda.current_stream()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        yield
        b.record(s)
        self.pairs.append((a, b))

    def elapsed_ms(self) -> float:
        total = 0.0
        for a, b in self.pairs:
            b.synchronize()
            total += a.elapsed_time(b)
        return total

    def reset(self):
        self.pairs = []
