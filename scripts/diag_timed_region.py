#!/usr/bin/env python3
"""Where the fixed cost of a short timed region goes (bench.py's K=20 region at N=1): the exact bench sequence
(barrier + sync, one FedAvg round of K steps, sync + barrier + sync) repeated, with hipEvents before the first and
after the last kernel, host timestamps after the launch call and after each sync.

    python scripts/diag_timed_region.py [K=20] [reps=9]
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer  # noqa: E402


def main(K=20, reps=9):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(1337)
    x = torch.randn(20000, 500, generator=g, device=dev)
    y = torch.zeros(20000, dtype=torch.long, device=dev)
    torch.manual_seed(1234)
    tr = FusedTinyTrainer(TinyECG().to(dev), x, y, 256, 50, seed=4321)
    tr.run_round(5, reset_loss=False)
    tr.prepare([K])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    from crossscale_ecg.ops import _lib
    raw = _lib._raw_stream
    rows = {"graph": [], "graph_slowstream": [], "graph_spin": [], "eager": []}
    for r in range(reps):
        for mode in rows:  # interleaved: same box state for all
            tr.use_graph = mode != "eager"
            _lib._raw_stream = None if mode == "graph_slowstream" else raw  # torch Stream object per launch
            tr.prepare_round(K, reset_loss=False)  # batches staged outside the timing (bench: behind the warmup)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            e0.record()
            tr.launch_round(K)
            t1 = time.perf_counter()
            e1.record()
            if mode == "graph_spin":  # poll the end event (no blocking wait), then the synchronize
                while not e1.query():
                    pass
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            span = e0.elapsed_time(e1) * 1e3
            rows[mode].append(((t1 - t0) * 1e6, (t2 - t0) * 1e6, (t3 - t0) * 1e6, span))
            c = rows[mode][-1]
            print(f"rep {r} {mode:16s}: launch call {c[0]:7.1f} us  sync1 {c[1]:7.1f}  sync2 {c[2]:7.1f}  gpu span "
                  f"{span:7.1f} us  -> wall/step {c[2] / K:6.2f}  span/step {span / K:6.2f}", flush=True)
    for mode, rr in rows.items():
        med = [statistics.median(c) for c in zip(*rr)]
        print(f"median {mode:16s}: launch call {med[0]:.1f} us, wall {med[2]:.1f} us, gpu span {med[3]:.1f} us, "
              f"fixed {med[2] - med[3]:.1f} us ({(med[2] - med[3]) / K:.2f} us/step at K={K}), "
              f"wall/step {med[2] / K:.2f} us")
    tr.close()


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:]]
    main(*a)
