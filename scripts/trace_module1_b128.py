#!/usr/bin/env python3
"""Module 1, B=128: where does A3's extra compute_ms go?  

``run``: A0 (random sampler, pageable) and A3 (contiguous, pin_memory=True, non_blocking) interleaved, each step's
compute (the eager Tiny1D train step + synchronize, bench/module1._Compute, the same step measure_step times) inside
a roctx range "A0/compute" / "A3/compute"; the training thread pinned to one CPU in both (as run_locality does).
Run it under

    rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d <dir> -o t -- \
        python3 scripts/trace_module1_b128.py run

``parse <dir>``: per configuration, medians over the compute ranges of: range wall time, GPU busy time of the
kernels that ran inside it, number of kernels, host time inside HIP launch calls, and the longest host gap between
consecutive HIP calls.  If GPU busy time and the launch calls' own time match between A0 and A3 while the wall and
the host gaps differ, the inflation is host-side scheduling of the launching thread, not the data path.
"""
import csv
import glob
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(iters=60, reps=3):
    import gc
    import tempfile

    import torch
    from torch.utils.data import DataLoader, RandomSampler, SequentialSampler

    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.bench.module1 import _Compute, _pin_threads, _sync, split_cpus
    from crossscale_ecg.data.dataset import ShardDataset
    from crossscale_ecg.data.shards import ensure_synthetic_shards
    from crossscale_ecg.utils import profiling

    dev = torch.device("cuda")
    ds = ShardDataset(ensure_synthetic_shards(tempfile.mkdtemp(prefix="ecg_tr_"), 20000, shard_size=8192))
    B, L = 128, ds.x.shape[1]
    step = _Compute(dev, "torch", B, L)
    pin_cpus = split_cpus()
    for _ in range(reps):
        for name, contiguous, pin, nb in (("A0", False, False, False), ("A3", True, True, True)):
            dl = DataLoader(ds, batch_size=B, sampler=SequentialSampler(ds) if contiguous else RandomSampler(ds),
                            num_workers=4, pin_memory=pin, drop_last=True, persistent_workers=True)
            it = iter(dl)
            prev = _pin_threads(it, pin_cpus)
            try:
                for i in range(iters + 5):
                    xc, yc = next(it)
                    _sync(dev)
                    x, y = xc.to(dev, non_blocking=nb), yc.to(dev, non_blocking=nb)
                    _sync(dev)
                    if i < 5:
                        step(x, y)
                        _sync(dev)
                        continue
                    with profiling.range(f"{name}/compute"):
                        step(x, y)
                        _sync(dev)
            finally:
                if prev is not None:
                    os.sched_setaffinity(0, prev)
            del it, dl
            gc.collect()
    print("done", flush=True)


def _rows(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def parse(d):
    markers = _rows(d, "*marker_api_trace.csv")
    kernels = _rows(d, "*kernel_trace.csv")
    hip = _rows(d, "*hip_api_trace.csv")
    ranges = [(m.get("Function") or m.get("Marker_Name") or "", int(m["Start_Timestamp"]), int(m["End_Timestamp"]))
              for m in markers]
    ranges = [r for r in ranges if r[0].endswith("/compute")]
    ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"])) for k in kernels)
    launches = sorted((int(h["Start_Timestamp"]), int(h["End_Timestamp"]), h.get("Function", ""))
                      for h in hip)
    out = {}
    for name, t0, t1 in ranges:
        kin = [(a, b) for a, b in ks if a >= t0 and b <= t1]
        busy = sum(b - a for a, b in kin)
        calls = [(a, b, f) for a, b, f in launches if a >= t0 and b <= t1]
        lt = sum(b - a for a, b, f in calls if "Launch" in f)
        gaps = [calls[i + 1][0] - calls[i][1] for i in range(len(calls) - 1)]
        out.setdefault(name.split("/")[0], []).append(
            ((t1 - t0) / 1e3, busy / 1e3, len(kin), lt / 1e3, (max(gaps) if gaps else 0) / 1e3,
             sum(gaps) / 1e3, len(calls)))
    print("per compute range, medians (us): wall | GPU kernel busy | kernels | host in launch calls | "
          "longest host gap | summed host gaps between HIP calls | HIP calls")
    for name, v in sorted(out.items()):
        med = [statistics.median(c) for c in zip(*v)]
        print(f"  {name}: n={len(v):3d}  wall {med[0]:8.1f}  gpu {med[1]:7.1f}  kernels {med[2]:4.0f}  launch "
              f"{med[3]:7.1f}  max-gap {med[4]:7.1f}  gaps {med[5]:7.1f}  calls {med[6]:4.0f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        parse(sys.argv[2])
