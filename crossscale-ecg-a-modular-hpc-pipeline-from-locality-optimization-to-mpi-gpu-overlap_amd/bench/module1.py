"""Module 1: data-locality benchmark (A0-A4) on MI355X.

Reference: Module_1/bench_locality.py (A0-A3, ``measure_step``) and
Module_1/train_ecg_labl(EXPERIMENTAL).py (A4 ``bench_labl``).  Configurations:

  A0_baseline          random sampler, pageable host batches, blocking H2D
  A1_contiguous        contiguous (sequential) sampler            <- the reference's A0 == A1 bug is fixed
  A2_contig_pinned     + pinned host batches
  A3_contig_pinned_nb  + non_blocking H2D
  A4_LABL              C++ mmap reader -> hipHostMalloc slab ring (producer thread) -> hipMemcpyAsync on a
                       copy stream, double-buffered against compute, event-fenced slab reuse, z-score
  A5_GPU_RESIDENT      whole shard resident in HBM (the Module-3 path; no per-step H2D)

Per-step breakdown (data_ms / h2d_ms / compute_ms) is measured like the reference (sync-bracketed
wall-clock).  ``step_ms`` is the measured wall time per step; for A0-A3 it equals the sum of the parts
(the parts are serialised by syncs, as in bench_locality.py:43-71), for A4 it is smaller because the
next batch's fill and copy overlap the current batch's compute.
``samples_per_s = (samples/iters) / (step_ms/1e3)`` (bench_locality.py:73-74).
``compute`` is the reference eager step (TinyECG fwd/CE/bwd/SGD lr 1e-2) or, with ``compute="fused"``,
the fused HIP step fed from the same device batch buffer (one native call enqueues the step kernel and the
reduce+SGD kernel, ~12 us of GPU time): with the ~0.6 ms of Python launches of the eager step gone, the A0-A3
comparison is one of the data path alone.  Its rows go to ``*_fused.csv`` next to the
reference-faithful eager rows.
"""
from __future__ import annotations

import gc
import os
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader, RandomSampler, SequentialSampler

from ..utils.timing import warm_until_stable

from ..data.dataset import ShardDataset
from ..data.shards import ensure_synthetic_shards, list_shards, shard_header
from ..models.tiny_ecg import TinyECG
from ..utils.csvio import LOCALITY_COLUMNS, LABL_COLUMNS, write_csv

CONFIGS = [
    ("A0_baseline", False, False, False),
    ("A1_contiguous", True, False, False),
    ("A2_contig_pinned", True, True, False),
    ("A3_contig_pinned_nb", True, True, True),
]


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class _Compute:
    """One training step on a device batch x [B,1,L], y [B]."""

    def __init__(self, dev, kind: str, B: int, L: int):
        self.dev, self.kind = dev, kind
        self.model = TinyECG().to(dev)
        if kind == "fused":
            from ..ops.fused_tiny import slab_stride
            self.flat = self.model.flatten_parameters()
            self.mom = torch.zeros_like(self.flat)
            self.slab = torch.empty((B, slab_stride(2)), device=dev)
            self.loss = torch.zeros(1, device=dev)
        else:
            self.opt = torch.optim.SGD(self.model.parameters(), lr=1e-2)

    def __call__(self, x: torch.Tensor, y: torch.Tensor):
        if self.kind == "fused":
            from ..ops import _lib
            x2 = x.reshape(x.shape[0], -1)
            y32 = y.to(torch.int32)
            st = _lib.kernels().ecg_tiny_train_step(x2.data_ptr(), x2.shape[1], x2.stride(0), None, y32.data_ptr(),
                                                    self.flat.data_ptr(), self.mom.data_ptr(), 2,
                                                    self.slab.data_ptr(), self.slab.shape[1], x2.shape[0],
                                                    self.loss.data_ptr(), 1e-2, 0.0, 0.0, 0, 0, None,
                                                    _lib.stream_ptr(self.dev))
            _lib.check(st, "ecg_tiny_train_step")
            return
        out = self.model(x)
        loss = F.cross_entropy(out, y)
        loss.backward()
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)


def split_cpus(cpus: Optional[Sequence[int]] = None):
    """(main-thread cpu, pin-thread cpu): two distinct CPUs of this process's affinity set (None if < 2)."""
    cpus = sorted(cpus if cpus is not None else os.sched_getaffinity(0))
    if len(cpus) < 2:
        return None
    return cpus[0], cpus[len(cpus) // 2]


def _pin_threads(it, pin_cpus) -> Optional[tuple]:
    """Put the calling (training) thread on CPU ``pin_cpus[0]`` - for EVERY configuration, so A0-A3 differ only in
    contiguity / pin_memory / non_blocking (the reference's comparison, bench_locality.py:111-116) - and, when the
    iterator has a pin-memory thread (A2/A3), that thread on ``pin_cpus[1]``, so the pinning copy does not compete
    with the launch-bound step for one core.  Call after the iterator (and its worker processes) exist, so the
    workers keep the inherited affinity.  Returns the calling thread's previous affinity (to restore), or None."""
    if pin_cpus is None:
        return None
    prev = os.sched_getaffinity(0)
    th = getattr(it, "_pin_memory_thread", None)
    if th is not None and getattr(th, "native_id", None) is not None:
        os.sched_setaffinity(th.native_id, {pin_cpus[1]})
    os.sched_setaffinity(0, {pin_cpus[0]})  # (Linux: pid 0 = the calling thread)
    return prev


def measure_step(dl: DataLoader, device, non_blocking: bool, iters: int = 50, compute: str = "torch",
                 pin_cpus: Optional[tuple] = None) -> Dict:
    """Reference ``measure_step`` (bench_locality.py:23-76): 5 warm-up steps, then timed data/H2D/compute.
    ``pin_cpus=(main, pin)``: the pin-memory thread and this thread on distinct CPUs (``split_cpus``)."""
    dev = torch.device(device)
    B = dl.batch_size
    L = dl.dataset.x.shape[1]
    step = _Compute(dev, compute, B, L)
    it = iter(dl)
    prev_aff = _pin_threads(it, pin_cpus)
    try:
        return _measure(dl, dev, non_blocking, iters, step, it, pin_cpus)
    finally:
        if prev_aff is not None:
            os.sched_setaffinity(0, prev_aff)


def _measure(dl, dev, non_blocking, iters, step, it, pin_cpus):

    def nxt():
        nonlocal it
        try:
            return next(it)
        except StopIteration:
            it = iter(dl)
            return next(it)

    def warm():
        xc, yc = nxt()
        step(xc.to(dev, non_blocking=non_blocking), yc.to(dev, non_blocking=non_blocking))

    warm_until_stable(warm, dev)  # >= 5 steps (reference), until no first-use compile remains
    data_ms = h2d_ms = comp_ms = 0.0
    total = 0
    it = iter(dl)
    _pin_threads(it, pin_cpus)  # the new iterator's pin thread
    t_all = time.perf_counter()
    for _ in range(iters):
        t0 = time.perf_counter()
        xc, yc = nxt()
        t1 = time.perf_counter()
        _sync(dev)
        th0 = time.perf_counter()
        x = xc.to(dev, non_blocking=non_blocking)
        y = yc.to(dev, non_blocking=non_blocking)
        _sync(dev)
        th1 = time.perf_counter()
        step(x, y)
        _sync(dev)
        t3 = time.perf_counter()
        data_ms += (t1 - t0) * 1e3
        h2d_ms += (th1 - th0) * 1e3
        comp_ms += (t3 - th1) * 1e3
        total += x.shape[0]
    wall = (time.perf_counter() - t_all) * 1e3 / iters
    sps = (total / iters) / (wall / 1e3)
    return dict(data_ms=data_ms / iters, h2d_ms=h2d_ms / iters, compute_ms=comp_ms / iters, step_ms=wall,
                samples_per_s=sps)


def bench_labl(shard_paths: Sequence[str], batch_size: int, iters: int, normalize: bool, device,
               compute: str = "torch", num_slots: int = 4) -> Dict:
    """A4: native LABL prefetcher + copy-stream H2D double buffer (reference bench_labl, :23-94).
    ``shard_paths`` is a list of shard files or, as in the reference, a glob string."""
    from ..ops.native_io import NativePrefetcher
    if isinstance(shard_paths, str):
        import glob as _glob
        shard_paths = sorted(_glob.glob(shard_paths))
        if not shard_paths:
            raise FileNotFoundError("bench_labl: no shards match the glob")
    dev = torch.device(device)
    pf = NativePrefetcher(shard_paths, batch_size, num_slots=num_slots, normalize=normalize,
                          pinned=dev.type == "cuda", loop=True)
    L = pf.L
    step = _Compute(dev, compute, batch_size, L)
    y = torch.zeros(batch_size, dtype=torch.long, device=dev)  # labels allocated once (reference re-pinned per step)
    bufs = [torch.empty((batch_size, 1, L), device=dev) for _ in range(2)]
    copy = torch.cuda.Stream(dev) if dev.type == "cuda" else None
    main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    ready = [None, None]
    consumed = [None, None]  # compute that last read bufs[k] (WAR fence for the next copy into it)
    pf.start()

    def stage(i):
        """Fill-wait + async H2D of the next slab into bufs[i%2]; returns (n, wait_ms)."""
        t0 = time.perf_counter()
        r = pf.next_batch_cpu()
        wait = (time.perf_counter() - t0) * 1e3
        slot, view, _fill = r
        n = view.shape[0]
        if dev.type == "cuda":
            if consumed[i % 2] is not None:
                copy.wait_event(consumed[i % 2])  # WAR: the compute that read this buffer must be done
            pf.h2d(slot, n, bufs[i % 2], copy)
            ev = torch.cuda.Event()
            ev.record(copy)
            ready[i % 2] = ev
        else:
            bufs[i % 2][:n].copy_(view)
            pf.recycle(slot)
        return n, wait

    try:
        wi = [0]

        def warm():  # warm-up step (>= 5, until stable)
            i = wi[0]
            wi[0] += 1
            n, _ = stage(i)
            if main is not None:
                main.wait_event(ready[i % 2])
            step(bufs[i % 2][:n], y[:n])
            if main is not None:
                consumed[i % 2] = torch.cuda.Event()
                consumed[i % 2].record(main)

        warm_until_stable(warm, dev)
        # The producer hands out each shard's tail as a short batch (n = windows % B); a new batch shape is a new
        # MIOpen problem whose first call runs the solver search (~0.2 s).  Round 1 timed that once at B=256 (its
        # 78-batch epoch put the 32-window tail inside the 100 timed steps: compute_ms 2.6-3.1 ms vs 0.75).  Warm
        # every tail shape here, outside the timing.
        for n_tail in sorted({shard_header(p)[0] % batch_size for p in shard_paths} - {0}):
            for _ in range(3):
                step(bufs[0][:n_tail], y[:n_tail])
        _sync(dev)
        data_ms = h2d_ms = comp_ms = 0.0
        total = 0
        n_next, w = stage(0)
        data_ms += w
        t_all = time.perf_counter()
        for i in range(iters):
            n = n_next
            if main is not None:
                th = time.perf_counter()
                main.wait_event(ready[i % 2])
                h2d_ms += (time.perf_counter() - th) * 1e3
            tc = time.perf_counter()
            step(bufs[i % 2][:n], y[:n])  # enqueue compute of batch i
            if main is not None:
                consumed[i % 2] = torch.cuda.Event()
                consumed[i % 2].record(main)
            if i + 1 < iters:
                n_next, w = stage(i + 1)  # fill + copy batch i+1 while batch i computes
                data_ms += w
            _sync(dev)
            comp_ms += (time.perf_counter() - tc) * 1e3
            total += n
        wall = (time.perf_counter() - t_all) * 1e3 / iters
    finally:
        pf.close()
    return dict(step_ms=wall, samples_per_s=(total / iters) / (wall / 1e3), data_ms=data_ms / iters,
                h2d_ms=h2d_ms / iters, compute_ms=comp_ms / iters)


def bench_gpu_resident(shard_paths, batch_size, iters, device, compute="torch") -> Dict:
    from ..data.dataset import load_shards_to_gpu, make_gpu_batch_iter
    dev = torch.device(device)
    x, y = load_shards_to_gpu(shard_paths, dev)
    it = make_gpu_batch_iter(x, y, batch_size)
    step = _Compute(dev, compute, batch_size, x.shape[1])
    for _ in range(5):
        step(*next(it))
    _sync(dev)
    t0 = time.perf_counter()
    for _ in range(iters):
        step(*next(it))
    _sync(dev)
    wall = (time.perf_counter() - t0) * 1e3 / iters
    return dict(step_ms=wall, samples_per_s=batch_size / (wall / 1e3), data_ms=0.0, h2d_ms=0.0, compute_ms=wall)


SPREAD_COLUMNS = ["samples_per_s_q1", "samples_per_s_q3", "reps"]


def _median_row(cells: List[Dict]) -> Dict:
    """Median of every timing column over the repetitions of one (config, batch) cell, plus the interquartile
    range of samples/s."""
    out = dict(cells[0])
    for k in ("data_ms", "h2d_ms", "compute_ms", "step_ms", "samples_per_s"):
        out[k] = float(np.median([c[k] for c in cells]))
    sps = [c["samples_per_s"] for c in cells]
    out["samples_per_s_q1"], out["samples_per_s_q3"] = (float(v) for v in np.percentile(sps, [25, 75]))
    out["reps"] = len(cells)
    return out


def run_locality(shard_dir: str, batch_sizes: List[int], iters: int = 100, num_workers: int = 4,
                 device: Optional[str] = None, compute: str = "torch", results_dir: str = "results",
                 n_windows: int = 20000, labl: bool = True, normalize: bool = True, reps: int = 1,
                 pin_thread: bool = False, reps_large: Optional[int] = None) -> List[Dict]:
    """A0-A5 per batch size.  ``reps`` > 1: every (config, batch) cell is measured ``reps`` times, the
    configurations interleaved within each repetition (A0 A1 A2 A3 A4 A5, A0 A1 ...), and the CSV holds the
    median of each column plus the samples/s interquartile range (``samples_per_s_q1/q3``, ``reps``).
    ``pin_thread``: the training thread of every A0-A3 configuration runs on one fixed CPU, and the pinned
    configurations' pin-memory thread on another (pinning only A2/A3 mixed thread placement into the
    A3-vs-A0 comparison).  ``reps_large``: repetitions for batch sizes >= 512 (default ``reps``)."""
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    paths = ensure_synthetic_shards(shard_dir, n_windows, shard_size=8192) if not list_shards(shard_dir) \
        else list_shards(shard_dir)
    ds = ShardDataset(paths)
    pin_cpus = split_cpus() if pin_thread else None
    rows, labl_rows = [], []
    for bs in batch_sizes:
        cells: Dict[str, List[Dict]] = {}
        n_reps = reps_large if (reps_large and bs >= 512) else reps
        for rep in range(max(1, n_reps)):
            for name, contiguous, pin, nb in CONFIGS:
                sampler = SequentialSampler(ds) if contiguous else RandomSampler(ds)
                dl = DataLoader(ds, batch_size=bs, sampler=sampler, num_workers=num_workers,
                                pin_memory=pin and dev.type == "cuda", drop_last=True,
                                persistent_workers=num_workers > 0)
                st = measure_step(dl, dev, non_blocking=nb, iters=iters, compute=compute, pin_cpus=pin_cpus)
                # retire this loader's persistent worker processes (and its pin-memory thread) before the next
                # config is timed: left alive they prefetch beside it (the A4 B=256 outlier of round 1)
                del dl
                gc.collect()
                row = dict(config=name, batch_size=bs, pin_memory=pin, contiguous=contiguous, non_blocking=nb, **st)
                print(dict(rep=rep, **row), flush=True)
                cells.setdefault(name, []).append(row)
            if labl:
                st = bench_labl(paths, bs, iters, normalize, dev, compute=compute)
                r = dict(config="A4_LABL", batch_size=bs, pin_memory=True, contiguous=True, non_blocking=True, **st)
                print(dict(rep=rep, **r), flush=True)
                cells.setdefault("A4_LABL", []).append(r)
            if dev.type == "cuda":
                st = bench_gpu_resident(paths, bs, iters, dev, compute=compute)
                r = dict(config="A5_GPU_RESIDENT", batch_size=bs, pin_memory=False, contiguous=False,
                         non_blocking=False, **st)
                print(dict(rep=rep, **r), flush=True)
                cells.setdefault("A5_GPU_RESIDENT", []).append(r)
        for name, cl in cells.items():
            row = _median_row(cl)
            rows.append(row)
            if name == "A4_LABL":
                labl_rows.append(row)
    os.makedirs(results_dir, exist_ok=True)
    sfx = "" if compute == "torch" else f"_{compute}"
    write_csv(os.path.join(results_dir, f"part1_locality_results{sfx}.csv"), rows, LOCALITY_COLUMNS + SPREAD_COLUMNS)
    if labl_rows:
        write_csv(os.path.join(results_dir, f"part1_labl_results{sfx}.csv"), labl_rows, LABL_COLUMNS + SPREAD_COLUMNS)
    return rows
