"""Pseudo-federated (independent per-rank) training benchmark: G0 baseline vs G1 overlap+AMP.

Reference: Module_3/part3_mpi_gpu_train.py
  * ``run_baseline_gpu`` (:100-184)  G0: fp32, per-step sync, GPU-resident batches
  * ``run_overlap_gpu``  (:306-412)  G1: AMP + one-batch lookahead (no real stream in the reference)
  * dead string-literal design (:187-305): pinned DataLoader + ``h2d_stream`` double buffer -> implemented
    here for real as ``run_stream_overlap`` (config ``G1_stream_overlap``)
  * ``main`` (:420-528): assign shards, load to GPU, run G0 then G1, gather BenchStats, rank 0 appends CSV.
Defects fixed: data_ms is actually accumulated, ``--data-root`` is honoured, G0 and G1 get
separate batch iterators, the G1 lookahead gather runs on a side stream and is genuinely overlapped.
"""
from __future__ import annotations

import time
from typing import Iterator, Optional, Tuple

import torch
import torch.nn.functional as F

from ..utils.csvio import BenchStats
from ..utils.timing import warm_until_stable


def _sync(device):
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)


def _world_size() -> int:
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def run_baseline_gpu(model, batch_iter: Iterator, device, steps: int, rank: int, batch_size: int,
                     lr: float = 1e-2, log_every: int = 10, warmup: int = 5) -> BenchStats:
    """G0: fp32, default stream, no overlap, sync every step (reference semantics)."""
    device = torch.device(device)
    model = model.to(device)
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9)
    model.train()
    def warm():  # untimed: MIOpen solver search / first-use kernel compiles (not in the reference)
        x, y = next(batch_iter)
        F.cross_entropy(model(x), y).backward()
        opt.zero_grad(set_to_none=True)

    warm_until_stable(warm, device, min_steps=warmup)
    data_ms = compute_ms = step_ms = 0.0
    n_samples = n_steps = 0
    while n_steps < steps:
        t0 = time.perf_counter()
        if rank == 0 and log_every and n_steps % log_every == 0:
            print(f"[G0][rank {rank}] step {n_steps}/{steps}", flush=True)
        x, y = next(batch_iter)
        _sync(device)
        t1 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        _sync(device)
        t2 = time.perf_counter()
        data_ms += (t1 - t0) * 1e3
        compute_ms += (t2 - t1) * 1e3
        step_ms += (t2 - t0) * 1e3
        n_samples += x.size(0)
        n_steps += 1
    avg = step_ms / max(1, n_steps)
    return BenchStats("G0_baseline_GPU_CACHE", _world_size(), rank, batch_size, n_steps, data_ms / n_steps, 0.0,
                      compute_ms / n_steps, avg, (n_samples / n_steps) / (avg / 1e3))


def run_overlap_gpu(model, batch_iter: Iterator, device, steps: int, rank: int, batch_size: int,
                    lr: float = 1e-2, amp_dtype=torch.bfloat16, log_every: int = 10, warmup: int = 5) -> BenchStats:
    """G1: AMP (bf16 by default) + lookahead: batch i+1's device gather is enqueued on a side stream while
    batch i computes on the main stream (reference did the lookahead in Python only)."""
    device = torch.device(device)
    if device.type != "cuda":
        raise RuntimeError("Overlap config requires a GPU")
    model = model.to(device)
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9)
    scaler = torch.amp.GradScaler("cuda") if amp_dtype == torch.float16 else None
    side = torch.cuda.Stream(device)
    main = torch.cuda.current_stream(device)
    model.train()
    def warm():  # untimed warm-up (MIOpen bf16 solver search / first-use compiles)
        x, y = next(batch_iter)
        with torch.autocast("cuda", dtype=amp_dtype):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.zero_grad(set_to_none=True)

    warm_until_stable(warm, device, min_steps=warmup)
    data_ms = compute_ms = step_ms = 0.0
    n_samples = n_steps = 0
    t_d0 = time.perf_counter()
    with torch.cuda.stream(side):
        x_prev, y_prev = next(batch_iter)
    ready = torch.cuda.Event()
    ready.record(side)
    data_ms += (time.perf_counter() - t_d0) * 1e3
    while n_steps < steps:
        t0 = time.perf_counter()
        if rank == 0 and log_every and n_steps % log_every == 0:
            print(f"[G1][rank {rank}] step {n_steps}/{steps}", flush=True)
        main.wait_event(ready)
        cur_x, cur_y = x_prev, y_prev
        cur_x.record_stream(main)
        cur_y.record_stream(main)
        td = time.perf_counter()
        with torch.cuda.stream(side):  # prefetch next batch (overlaps the compute below)
            side.wait_stream(main)
            x_prev, y_prev = next(batch_iter)
            ready = torch.cuda.Event()
            ready.record(side)
        data_ms += (time.perf_counter() - td) * 1e3
        t1 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=amp_dtype):
            loss = F.cross_entropy(model(cur_x), cur_y)
        if scaler is not None:
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
        else:
            loss.backward()
            opt.step()
        _sync(device)
        t2 = time.perf_counter()
        compute_ms += (t2 - t1) * 1e3
        step_ms += (t2 - t0) * 1e3
        n_samples += cur_x.size(0)
        n_steps += 1
    avg = step_ms / max(1, n_steps)
    return BenchStats("G1_overlap_amp", _world_size(), rank, batch_size, n_steps, data_ms / n_steps, 0.0,
                      compute_ms / n_steps, avg, (n_samples / n_steps) / (avg / 1e3))


def run_fused_gpu(model, x_gpu, y_gpu, device, steps: int, rank: int, batch_size: int, lr: float = 1e-2,
                  seed: Optional[int] = None, precision: str = "bf16") -> BenchStats:
    """The fused HIP step (``precision`` bf16: G1, fp32: the native G0): all ``steps`` replayed from one native
    hipGraph, one sync at the end.  The graph for exactly ``steps`` steps is captured and uploaded - and its
    kernels warmed by one replay that ``prepare`` rolls back - before the timing starts."""
    from ..ops.fused_tiny import FusedTinyTrainer
    tr = FusedTinyTrainer(model, x_gpu, y_gpu, batch_size, steps, lr=lr, momentum=0.9, seed=seed,
                          precision=precision)
    tr.prepare([steps])
    _sync(device)
    t0 = time.perf_counter()
    tr.run_round(steps)
    _sync(device)
    ms = (time.perf_counter() - t0) * 1e3
    tr.close()
    avg = ms / steps
    name = "G1_fused_hip_graph" if precision == "bf16" else "G0_fused_hip_fp32"
    return BenchStats(name, _world_size(), rank, batch_size, steps, 0.0, 0.0, avg, avg, batch_size / (avg / 1e3))


def run_stream_overlap(model, dl, device, steps: int, rank: int, batch_size: int, lr: float = 1e-2,
                       amp_dtype=torch.bfloat16) -> BenchStats:
    """The reference's intended (dead-code, part3_mpi_gpu_train.py:187-305) design, implemented: pinned host
    batches, H2D of batch i+1 on ``h2d_stream`` while batch i computes, ``wait_stream`` + double buffer."""
    device = torch.device(device)
    model = model.to(device)
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9)
    h2d = torch.cuda.Stream(device)
    main = torch.cuda.current_stream(device)
    it = iter(dl)

    def fetch():
        nonlocal it
        try:
            return next(it)
        except StopIteration:
            it = iter(dl)
            return next(it)

    data_ms = h2d_ms = compute_ms = step_ms = 0.0
    n_samples = n_steps = 0
    xc, yc = fetch()
    with torch.cuda.stream(h2d):
        x_next = xc.to(device, non_blocking=True)
        y_next = yc.to(device, non_blocking=True)
    while n_steps < steps:
        t0 = time.perf_counter()
        main.wait_stream(h2d)
        x, y = x_next, y_next
        x.record_stream(main)
        y.record_stream(main)
        td = time.perf_counter()
        xc, yc = fetch()
        t_h = time.perf_counter()
        with torch.cuda.stream(h2d):
            x_next = xc.to(device, non_blocking=True)
            y_next = yc.to(device, non_blocking=True)
        t1 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=amp_dtype):
            loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        _sync(device)
        t2 = time.perf_counter()
        data_ms += (t_h - td) * 1e3
        h2d_ms += (t1 - t_h) * 1e3
        compute_ms += (t2 - t1) * 1e3
        step_ms += (t2 - t0) * 1e3
        n_samples += x.size(0)
        n_steps += 1
    avg = step_ms / n_steps
    return BenchStats("G1_stream_overlap", _world_size(), rank, batch_size, n_steps, data_ms / n_steps,
                      h2d_ms / n_steps, compute_ms / n_steps, avg, (n_samples / n_steps) / (avg / 1e3))
