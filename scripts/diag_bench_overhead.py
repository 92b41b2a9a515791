#!/usr/bin/env python3
"""Where does the fixed (per timed region) overhead of a short bench.py run go?

Times, in one process after warm-up, the FedAvg round plan of K steps for several K (5 repetitions each) and
the pieces of a round in isolation: the index-table fill, a graph replay of n steps, a bare synchronize.
"""
from __future__ import annotations

import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(1337)
    x = torch.randn(20000, 500, generator=g, device=dev)
    y = torch.zeros(20000, dtype=torch.long, device=dev)
    torch.manual_seed(1234)
    m = TinyECG().to(dev)
    tr = FusedTinyTrainer(m, x, y, 256, 50, seed=4321)
    tr.prepare([1, 5, 20, 50])
    for _ in range(4):
        tr.run_round(50)
    torch.cuda.synchronize()

    def timed(fn, reps=7):
        out = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            out.append((time.perf_counter() - t0) * 1e6)
        return statistics.median(out), min(out)

    def plan(k):
        def f():
            sizes = [50] * (k // 50) + ([k % 50] if k % 50 else [])
            for i, n in enumerate(sizes):  # staged like bench.py: next round's batches behind this round
                tr.run_round(n, reset_loss=False, next_n=sizes[i + 1] if i + 1 < len(sizes) else None)
        return f

    print("bare synchronize: median %.1f us  min %.1f us" % timed(lambda: None))
    print("index fill (20 rows): median %.1f us  min %.1f us" % timed(lambda: tr.sampler.fill(tr.idx_stage[:20])))
    for n in (1, 5, 20, 50):
        med, mn = timed(lambda: (tr.prepare_round(n, reset_loss=False), tr.launch_round(n)))
        print(f"round n={n:3d} (fill + replay): median {med:8.1f} us  min {mn:8.1f} us  -> {med / n:6.2f} us/step")
    for k in (20, 50, 100, 500):
        med, mn = timed(plan(k))
        print(f"plan K={k:4d}: median {med:8.1f} us  min {mn:8.1f} us  -> {med / k:6.2f} us/step (min {mn / k:6.2f})")
    # replay only, batches staged outside the timing (as bench.py's first timed round): host wall, time for the
    # launch call to return, and the GPU span between events recorded just before / after the replay
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for n in (1, 2, 20, 50):
        wall, call, span = [], [], []
        for _ in range(9):
            tr.prepare_round(n, reset_loss=False)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            t1 = time.perf_counter()
            tr.launch_round(n)
            t2 = time.perf_counter()
            e1.record()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            wall.append((t3 - t0) * 1e6)
            call.append((t2 - t1) * 1e6)
            span.append(e0.elapsed_time(e1) * 1e3)
        med = statistics.median
        print(f"replay n={n:3d}: wall {med(wall):8.1f} us  launch call {med(call):6.1f} us  "
              f"gpu span {med(span):8.1f} us  -> wall {med(wall) / n:6.2f} / span {med(span) / n:6.2f} us/step")
    # the same kernels enqueued one by one from a C++ loop (no graph)
    from crossscale_ecg.ops import _lib
    lib = _lib.kernels()
    stream = _lib.stream_ptr(dev)
    for n in (1, 2, 20, 50):
        wall, call = [], []
        for _ in range(9):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st = lib.ecg_tiny_train_steps_pf(tr.x.data_ptr(), tr.x.shape[1], tr.x.stride(0), tr.idx_table.data_ptr(),
                                             tr.y32.data_ptr(), tr.params.data_ptr(), tr.mom.data_ptr(), tr.nc,
                                             tr.slab.data_ptr(), tr.stride, tr.B, n, tr.loss_acc.data_ptr(), tr.lr,
                                             tr.momentum, tr.wd, int(tr.nesterov), tr.wprep.data_ptr(), 0, stream)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            _lib.check(st, "ecg_tiny_train_steps_pf")
            wall.append((t2 - t0) * 1e6)
            call.append((t1 - t0) * 1e6)
        med = statistics.median
        print(f"eager C loop n={n:3d}: wall {med(wall):8.1f} us  enqueue {med(call):6.1f} us  "
              f"-> {med(wall) / n:6.2f} us/step")
    tr.close()


if __name__ == "__main__":
    main()
