"""Python face of the C++ Module-1 data path (csrc/io/shard_io.cpp).

* ``MappedShard``        - mmap'd shard (zero-copy numpy view), reference ``LABLShardedReader.open_shard``
                           (Module_1/labl_loader(EXPERIMENTAL).py:7-28).
* ``NativePrefetcher``   - C++ producer thread filling a ring of hipHostMalloc slabs; reference
                           ``PinnedRing`` + ``LABLPrefetcher`` (:30-136), same method names
                           (start / shutdown / next_batch_cpu / recycle) plus ``h2d`` (async copy on a
                           stream + event-fenced slab reuse).
* ``upload_shards``      - chunked pinned double-buffer upload for GPU-resident shards.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib


def available() -> bool:
    return _lib.io_available()


def _paths_array(paths: Sequence[str]):
    arr = (C.c_char_p * len(paths))(*[p.encode() for p in paths])
    return arr


class MappedShard:
    def __init__(self, path: str):
        lib = _lib.io_lib()
        self._h = C.c_void_p()
        n, l = C.c_int64(), C.c_int64()
        _lib.check(lib.ecg_shard_open(path.encode(), C.byref(self._h), C.byref(n), C.byref(l)), f"open {path}")
        self.N, self.L = n.value, l.value
        ptr = lib.ecg_shard_data(self._h)
        buf = (C.c_float * (self.N * self.L)).from_address(ptr) if self.N else None
        self.array = np.ctypeslib.as_array(buf).reshape(self.N, self.L) if buf is not None else \
            np.empty((0, self.L), np.float32)

    def close(self):
        if self._h.value:
            self.array = None
            _lib.io_lib().ecg_shard_close(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class NativePrefetcher:
    """Background C++ producer of [B, 1, L] batches in pinned (or plain, for CPU tests) host slabs."""

    def __init__(self, paths: Sequence[str], batch_size: int, num_slots: int = 4, normalize: bool = True,
                 pinned: Optional[bool] = None, loop: bool = False):
        if pinned is None:
            pinned = torch.cuda.is_available()
        self.lib = _lib.io_lib()
        self._paths = _paths_array(list(paths))
        self._h = C.c_void_p()
        L = C.c_int64()
        _lib.check(self.lib.ecg_prefetch_create(self._paths, len(paths), batch_size, num_slots, int(normalize),
                                                int(pinned), int(loop), C.byref(self._h), C.byref(L)),
                   "ecg_prefetch_create")
        self.B, self.L, self.num_slots, self.pinned = batch_size, L.value, num_slots, pinned
        self._views = []
        for s in range(num_slots):
            p = self.lib.ecg_prefetch_slot_ptr(self._h, s)
            arr = np.ctypeslib.as_array((C.c_float * (batch_size * self.L)).from_address(p))
            self._views.append(torch.from_numpy(arr).view(batch_size, 1, self.L))
        self.stop = False

    def start(self):
        _lib.check(self.lib.ecg_prefetch_start(self._h), "ecg_prefetch_start")

    def next_batch_cpu(self, timeout_ms: int = 100) -> Optional[Tuple[int, torch.Tensor, float]]:
        """(slot, batch_view [n,1,L], fill_ms) or None at end of data."""
        slot, n, ms = C.c_int(), C.c_int(), C.c_double()
        while True:
            st = self.lib.ecg_prefetch_next(self._h, timeout_ms, C.byref(slot), C.byref(n), C.byref(ms))
            if st == 5:  # timeout: keep polling unless shut down
                if self.stop:
                    return None
                continue
            if st == 6:
                return None
            if st == 4:
                raise _lib.NativeError(self.lib.ecg_prefetch_error(self._h).decode())
            _lib.check(st, "ecg_prefetch_next")
            return slot.value, self._views[slot.value][: n.value], float(ms.value)

    def recycle(self, slot: int, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Return a slab. With ``stream`` the slab is refilled only after work queued on it completes."""
        if stream is not None and self.pinned:
            _lib.check(self.lib.ecg_prefetch_recycle_after(self._h, slot, stream.cuda_stream), "recycle_after")
        else:
            _lib.check(self.lib.ecg_prefetch_recycle(self._h, slot), "recycle")

    def h2d(self, slot: int, n: int, dst: torch.Tensor, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Async copy of the slab's first n windows into dst (device, contiguous) then fenced recycle."""
        if not dst.is_cuda or not dst.is_contiguous() or dst.numel() < n * self.L or dst.dtype != torch.float32:
            raise ValueError("dst must be a contiguous float32 CUDA tensor with room for n windows")
        s = stream or torch.cuda.current_stream(dst.device)
        _lib.check(self.lib.ecg_prefetch_h2d(self._h, slot, n, dst.data_ptr(), s.cuda_stream), "ecg_prefetch_h2d")

    def shutdown(self):
        self.stop = True
        if self._h.value:
            self.lib.ecg_prefetch_shutdown(self._h)

    def close(self):
        if self._h.value:
            self.shutdown()
            self._views = []
            self.lib.ecg_prefetch_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def upload_shards(paths: Sequence[str], device, n_rows: int, L: int, chunk_rows: int = 32768,
                  threads: Optional[int] = None) -> torch.Tensor:
    """Upload the first ``n_rows`` windows of ``paths`` into a new device tensor [n_rows, L].

    ``threads`` host threads copy each chunk from the mmap'd shards into one of three pinned staging buffers
    while the previous chunk's DMA runs (default: the process's usable CPUs, at most 8)."""
    from ..utils import usable_cpus
    dev = torch.device(device)
    x = torch.empty((n_rows, L), dtype=torch.float32, device=dev)
    arr = _paths_array(list(paths))
    rows = C.c_int64()
    stream = torch.cuda.current_stream(dev)
    th = int(threads) if threads else max(1, min(8, usable_cpus()))
    _lib.check(_lib.io_lib().ecg_upload_shards_mt(arr, len(paths), n_rows, L, x.data_ptr(), chunk_rows, th,
                                                  stream.cuda_stream, C.byref(rows)), "ecg_upload_shards")
    if rows.value != n_rows:
        raise RuntimeError(f"uploaded {rows.value} rows, expected {n_rows}")
    return x
