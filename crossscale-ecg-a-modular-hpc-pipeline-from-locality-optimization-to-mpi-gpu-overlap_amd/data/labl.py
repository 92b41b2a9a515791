"""LABL (locality-aware batch loader) API under the reference's names, backed by the C++ data path.

Reference: ``Module_1/labl_loader(EXPERIMENTAL).py`` - a Python mmap reader (:7-28), a ring of pinned
slabs with free/full queues (:30-36) and a daemon-thread prefetcher (:38-136).  The reference file cannot be
imported (the parentheses in its name); this module is the importable equivalent.

* ``LABLShardedReader(paths).open_shard(path)`` yields ``(mm, base, N, L)`` exactly like the reference
  (``np.frombuffer(mm, np.float32, count=L, offset=base + i*L*4)`` reads window ``i``), but ``mm`` is a
  read-only memoryview of the C++ ``mmap`` + ``madvise(SEQUENTIAL)`` mapping (csrc/io/shard_io.cpp).
* ``PinnedRing(num_slots, batch_shape)`` - page-locked slabs plus free/full queues (reference fields
  ``slots``, ``q_free``, ``q_full``), for callers that drive their own producer.
* ``LABLPrefetcher(reader, batch_size, num_slots=4, normalize=True)`` - same constructor and methods
  (``start / shutdown / next_batch_cpu / recycle``) but the producer is a C++ ``std::thread`` filling
  ``hipHostMalloc`` slabs (float64-accumulated z-score as in :65-69); ``h2d`` adds the one-copy-per-batch
  upload on a stream with event-fenced slab reuse.  Batches never span shards (a short batch at each
  shard end, as in :91-95).  Difference from the reference, on purpose: a slab passed to
  ``recycle(slot, stream)`` is refilled only after the copy reading it completed (the reference recycles
  while its ``non_blocking`` copy may still be in flight), and ``loop=True`` restarts at the first shard.
"""
from __future__ import annotations

import ctypes as C
import queue
import weakref
from contextlib import contextmanager
from typing import Iterable, Optional, Sequence, Tuple

import torch

from ..ops import _lib
from ..ops.native_io import MappedShard, NativePrefetcher

HEADER_BYTES = 16


class LABLShardedReader:
    """Shard list + mmap opener (format ``[int64 N][int64 L][float32 N*L]``)."""

    def __init__(self, shard_paths: Iterable[str]):
        self.paths = list(shard_paths)

    @contextmanager
    def open_shard(self, path: str):
        m = MappedShard(path)
        m.array = None
        ptr = _lib.io_lib().ecg_shard_data(m._h)
        size = HEADER_BYTES + m.N * m.L * 4
        # the C++ mapping covers the whole file from offset 0; data() is mapping + 16
        raw = (C.c_char * size).from_address(ptr - HEADER_BYTES)
        # Arrays made from ``mm`` (np.frombuffer) keep ``raw`` alive: unmap only when the last one is gone,
        # so a view that outlives the ``with`` block never dangles.
        weakref.finalize(raw, m.close)
        mm = memoryview(raw).cast("B").toreadonly()
        try:
            yield mm, HEADER_BYTES, int(m.N), int(m.L)
        finally:
            mm.release()
            del mm, raw


class PinnedRing:
    """``num_slots`` page-locked slabs shaped like a batch, with free / full slot queues."""

    def __init__(self, num_slots: int, batch_shape: Tuple[int, ...], dtype: torch.dtype = torch.float32):
        pin = torch.cuda.is_available()
        self.slots = [torch.empty(batch_shape, dtype=dtype, pin_memory=pin) for _ in range(num_slots)]
        self.q_free: "queue.Queue[int]" = queue.Queue()
        self.q_full: "queue.Queue[tuple]" = queue.Queue()
        for i in range(num_slots):
            self.q_free.put(i)


class LABLPrefetcher:
    """Reference-compatible prefetcher over the native C++ producer (see module docstring)."""

    def __init__(self, reader: LABLShardedReader, batch_size: int, num_slots: int = 4, normalize: bool = True,
                 loop: bool = False, pinned: Optional[bool] = None):
        if not reader.paths:
            raise ValueError("LABLPrefetcher: reader has no shard paths")
        self.reader = reader
        self.B = batch_size
        self.normalize = normalize
        self._native = NativePrefetcher(reader.paths, batch_size, num_slots=num_slots, normalize=normalize,
                                        pinned=pinned, loop=loop)
        self.L = self._native.L
        self.num_slots = num_slots

    @property
    def stop(self) -> bool:
        return self._native.stop

    def start(self) -> None:
        self._native.start()

    def shutdown(self) -> None:
        self._native.shutdown()

    def next_batch_cpu(self):
        """``(slot, batch_view [n,1,L], fill_ms)`` or ``None`` at end of data / after shutdown."""
        return self._native.next_batch_cpu()

    def recycle(self, slot: int, stream: Optional["torch.cuda.Stream"] = None) -> None:
        self._native.recycle(slot, stream)

    def h2d(self, slot: int, n: int, dst: torch.Tensor, stream: Optional["torch.cuda.Stream"] = None) -> None:
        self._native.h2d(slot, n, dst, stream)

    def close(self) -> None:
        self._native.close()

    def __iter__(self):
        """Yield ``(batch_view, fill_ms)``; each slab is recycled when the next one is requested."""
        prev = None
        while True:
            if prev is not None:
                self.recycle(prev)
            got = self.next_batch_cpu()
            if got is None:
                return
            prev, batch, ms = got
            yield batch, ms


def iter_windows(paths: Sequence[str]):
    """Yield ``(path, N, L)`` for each shard (header only; cheap)."""
    r = LABLShardedReader(paths)
    for p in r.paths:
        with r.open_shard(p) as (_mm, _base, n, l):
            yield p, n, l
