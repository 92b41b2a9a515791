#!/usr/bin/env python3
"""Diagnose the A4_LABL per-batch-size anomaly (profiles/r1_modules/part1_locality_results.csv: B=256 ~3x slower
compute than B=128/512): per-piece wall times of the bench_labl loop (fill wait, H2D enqueue, compute enqueue,
synchronize), the compute alone on resident data, and hipEvent device times of the H2D and of the step."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.module1 import _Compute  # noqa: E402
from crossscale_ecg.data.shards import write_shard  # noqa: E402
from crossscale_ecg.ops.native_io import NativePrefetcher  # noqa: E402


def make_shards(shard_dir="/tmp/diag_labl_shards"):
    os.makedirs(shard_dir, exist_ok=True)
    rng = np.random.default_rng(1337)
    paths = []
    for i in range(2):
        p = os.path.join(shard_dir, f"ecg_{i:05d}.bin")
        if not os.path.exists(p):
            write_shard(p, rng.normal(0, 1, (32768, 500)).astype(np.float32))
        paths.append(p)
    return paths


def main(shard_dir="/tmp/diag_labl_shards"):
    paths = make_shards(shard_dir)
    dev = torch.device("cuda:0")
    for B in (128, 256, 512):
        for compute in ("torch", "fused"):
            pf = NativePrefetcher(paths, B, num_slots=4, normalize=True, pinned=True, loop=True)
            step = _Compute(dev, compute, B, 500)
            y = torch.zeros(B, dtype=torch.long, device=dev)
            buf = torch.empty((B, 1, 500), device=dev)
            copy = torch.cuda.Stream(dev)
            pf.start()
            t = {k: [] for k in ("fill", "h2d_enq", "wait", "step_enq", "sync", "h2d_dev", "step_dev")}
            try:
                for it in range(80):
                    t0 = time.perf_counter()
                    slot, view, _ = pf.next_batch_cpu()
                    t1 = time.perf_counter()
                    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                    e0.record(copy)
                    pf.h2d(slot, view.shape[0], buf, copy)
                    e1.record(copy)
                    t2 = time.perf_counter()
                    torch.cuda.current_stream().wait_event(e1)
                    t3 = time.perf_counter()
                    step(buf, y)
                    e2.record()
                    t4 = time.perf_counter()
                    torch.cuda.synchronize()
                    t5 = time.perf_counter()
                    if it >= 20:
                        for k, v in (("fill", t1 - t0), ("h2d_enq", t2 - t1), ("wait", t3 - t2), ("step_enq", t4 - t3),
                                     ("sync", t5 - t4)):
                            t[k].append(v * 1e3)
                        t["h2d_dev"].append(e0.elapsed_time(e1))
                        t["step_dev"].append(e1.elapsed_time(e2))
            finally:
                pf.close()
            med = {k: round(statistics.median(v), 4) for k, v in t.items()}
            # the same step on the same (resident) buffer, no loader
            for _ in range(10):
                step(buf, y)
            torch.cuda.synchronize()
            s0 = time.perf_counter()
            for _ in range(50):
                step(buf, y)
            torch.cuda.synchronize()
            alone = (time.perf_counter() - s0) * 1e3 / 50
            print(f"B={B} compute={compute} median ms: {med}  step alone {alone:.4f} ms", flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def trace_bench_labl(shard_dir="/tmp/diag_labl_shards"):
    """The real A4 loop (bench.module1.bench_labl) at B=128/256/512, then a torch.profiler trace of B=256:
    top device kernels and the host-side calls that wait."""
    from crossscale_ecg.bench.module1 import bench_labl
    paths = make_shards(shard_dir)
    dev = torch.device("cuda:0")
    for B in (128, 256, 512, 256):
        r = bench_labl(paths, B, 100, True, dev)
        print(f"bench_labl B={B}: " + ", ".join(f"{k} {v:.4f}" for k, v in r.items()), flush=True)
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        bench_labl(paths, 256, 40, True, dev)
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=15))
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=15))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "trace":
    trace_bench_labl()
