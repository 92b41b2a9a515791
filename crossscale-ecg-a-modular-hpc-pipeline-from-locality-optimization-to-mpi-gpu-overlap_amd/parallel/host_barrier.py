"""Single-node host barrier over shared memory (``csrc/io/host_barrier.cpp``) for timing brackets.

``bench.py`` brackets its timed region with barrier + synchronize on both sides.  On the RCCL backend
``dist.barrier`` is a one-element all-reduce plus a stream synchronisation: tens of microseconds at 8 ranks,
i.e. several percent of a 20-step TinyECG region (~240 us).  The ranks of a single-node job meet in a POSIX
shared-memory page instead (a sense-reversing counter, ~1 us): the closing barrier then measures when the
slowest rank finished, not the latency of a collective.  Same semantics as any barrier.

Used only when every rank of the job is on this node (``LOCAL_WORLD_SIZE == WORLD_SIZE``) and every rank
could map the segment (agreed over the process group at setup); otherwise it is ``dist.barrier``.
"""
from __future__ import annotations

import ctypes as C
import os
import secrets
from typing import Optional

import torch.distributed as dist

from ..ops import _lib
from .env import DistContext, barrier as dist_barrier


def _bind(lib) -> None:
    if getattr(lib, "_host_barrier_bound", False):
        return
    _lib._sig(lib, "ecg_host_barrier_open", [C.c_char_p, _lib.i32, _lib.i32, C.POINTER(_lib.vp)])
    _lib._sig(lib, "ecg_host_barrier_wait", [_lib.vp, _lib.i32])
    _lib._sig(lib, "ecg_host_barrier_close", [_lib.vp])
    _lib._sig(lib, "ecg_host_barrier_unlink", [_lib.vp])
    lib._host_barrier_bound = True


class HostBarrier:
    """``b()`` returns once every rank of the job called it (the n-th calls meet).  ``b.kind``: "shm", "dist"
    (process-group barrier) or "none" (single process)."""

    def __init__(self, ctx: DistContext, timeout_s: float = 300.0):
        self.ctx = ctx
        self.timeout_ms = int(timeout_s * 1000)
        self._h: Optional[C.c_void_p] = None
        self._lib = None
        self.kind = "none"
        if not ctx.distributed:
            return
        self.kind = "dist"
        local = int(os.environ.get("LOCAL_WORLD_SIZE", "-1"))
        if os.environ.get("ECG_HOST_BARRIER", "1") == "0" or local != ctx.world_size:
            return
        names = [f"/ecg_bar_{os.getpid()}_{secrets.token_hex(6)}" if ctx.rank == 0 else None]
        dist.broadcast_object_list(names, src=0)
        name = names[0]
        ok = self._open(name, create=ctx.rank == 0) if ctx.rank == 0 else True
        dist_barrier(ctx)  # the segment exists before any peer opens it
        if ctx.rank != 0:
            ok = self._open(name, create=False)
        oks = [None] * ctx.world_size
        dist.all_gather_object(oks, bool(ok))
        if all(oks):
            self.kind = "shm"
            if ctx.rank == 0:  # every rank holds its mapping: drop the name now, so a crash leaks nothing
                self._lib.ecg_host_barrier_unlink(self._h)
        else:  # every rank falls back together
            self._close_handle()

    def _open(self, name: str, create: bool) -> bool:
        try:
            lib = _lib.io_lib()
            _bind(lib)
            h = _lib.vp()
            rc = lib.ecg_host_barrier_open(name.encode(), self.ctx.world_size, int(create), C.byref(h))
            if rc != 0:
                return False
            self._lib, self._h = lib, h
            return True
        except Exception:
            return False

    def __call__(self) -> None:
        if self.kind == "shm":
            rc = self._lib.ecg_host_barrier_wait(self._h, self.timeout_ms)
            if rc != 0:
                raise RuntimeError(f"host barrier failed (code {rc}): a peer rank did not arrive within "
                                   f"{self.timeout_ms} ms")
        elif self.kind == "dist":
            dist_barrier(self.ctx)

    def _close_handle(self) -> None:
        if self._h is not None and self._lib is not None:
            self._lib.ecg_host_barrier_close(self._h)
        self._h = None

    def close(self) -> None:
        """Collective: every rank is done with the segment before the creator unlinks it."""
        if self.kind == "shm":
            dist_barrier(self.ctx)
        self._close_handle()
        self.kind = "none" if not self.ctx.distributed else "dist"
