#!/usr/bin/env python3
"""Module 1: does the DataLoader's pin-memory thread slow the launch-bound eager step?

Times the reference step breakdown (bench/module1.measure_step) for three loaders over the same shards,
interleaved over reps:
  A0        random sampler, pageable batches (reference baseline)
  A3        contiguous + pin_memory=True (torch's pin thread in this process) + non_blocking H2D
  A3_main   contiguous, pageable loader; the batch is pinned in the main thread inside the data timing
            (no pin thread running during compute) + non_blocking H2D
If A3's compute_ms sits above A0's and A3_main's does not, the pin thread's GIL/CPU share is what inflates
the compute of the ~0.7 ms launch-bound step.

    python scripts/diag_pin_thread.py [reps=3] [iters=100]
"""
import gc
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.utils.data import DataLoader, RandomSampler, SequentialSampler  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.module1 import measure_step  # noqa: E402
from crossscale_ecg.data.dataset import ShardDataset  # noqa: E402
from crossscale_ecg.data.shards import ensure_synthetic_shards  # noqa: E402


class MainThreadPin:
    """Iterable over a pageable DataLoader that pins each batch in the calling thread."""

    def __init__(self, dl):
        self.dl, self.batch_size, self.dataset = dl, dl.batch_size, dl.dataset

    def __iter__(self):
        for xc, yc in self.dl:
            yield xc.pin_memory(), yc.pin_memory()


def main(reps=3, iters=100):
    dev = torch.device("cuda")
    d = tempfile.mkdtemp(prefix="ecg_pin_")
    ds = ShardDataset(ensure_synthetic_shards(d, 20000, shard_size=8192))
    res = {}
    for r in range(reps):
        for bs in (64, 128, 256, 512):
            for name in ("A0", "A3", "A3_main"):
                contiguous = name != "A0"
                dl = DataLoader(ds, batch_size=bs, sampler=SequentialSampler(ds) if contiguous else RandomSampler(ds),
                                num_workers=4, pin_memory=name == "A3", drop_last=True, persistent_workers=True)
                src = MainThreadPin(dl) if name == "A3_main" else dl
                st = measure_step(src, dev, non_blocking=name != "A0", iters=iters)
                del dl, src
                gc.collect()
                res.setdefault((bs, name), []).append(st)
                print(f"rep {r} B={bs:3d} {name:8s}: data {st['data_ms']:.3f} h2d {st['h2d_ms']:.3f} "
                      f"compute {st['compute_ms']:.3f} step {st['step_ms']:.3f} ms  {st['samples_per_s']:.0f}/s",
                      flush=True)
    print("median over reps:")
    for (bs, name), sts in sorted(res.items()):
        med = {k: sorted(s[k] for s in sts)[len(sts) // 2] for k in sts[0]}
        print(f"B={bs:3d} {name:8s}: data {med['data_ms']:.3f} h2d {med['h2d_ms']:.3f} compute {med['compute_ms']:.3f} "
              f"step {med['step_ms']:.3f} ms  {med['samples_per_s']:.0f}/s")


if __name__ == "__main__":
    main(*[int(v) for v in sys.argv[1:]])
