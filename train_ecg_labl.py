#!/usr/bin/env python3
"""A4 LABL benchmark CLI (reference Module_1/train_ecg_labl(EXPERIMENTAL).py; its broken import is fixed).

    python train_ecg_labl.py --shards 'data/shards/ecg_*.bin' --batch-sizes 64 128 256 512 --iters 200
Uses the native C++ prefetcher (mmap -> hipHostMalloc ring -> hipMemcpyAsync on a copy stream).
Writes results/part1_labl_results.csv (config A4_LABL)."""
import argparse
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.module1 import bench_labl  # noqa: E402
from crossscale_ecg.data.shards import ensure_synthetic_shards  # noqa: E402
from crossscale_ecg.utils.csvio import LABL_COLUMNS, write_csv  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="data/shards/ecg_*.bin")
    ap.add_argument("--batch-sizes", nargs="+", type=int, default=[64, 128, 256, 512])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--device", default=None)
    ap.add_argument("--no-normalize", action="store_true")
    ap.add_argument("--compute", choices=["torch", "fused"], default="torch")
    ap.add_argument("--results-dir", default="results")
    a = ap.parse_args(argv)
    paths = sorted(glob.glob(a.shards))
    if not paths:
        paths = ensure_synthetic_shards(os.path.dirname(a.shards) or "data/shards", 20000, shard_size=8192)
    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    rows = []
    for bs in a.batch_sizes:
        st = bench_labl(paths, bs, a.iters, not a.no_normalize, dev, compute=a.compute)
        rows.append(dict(config="A4_LABL", batch_size=bs, **st))
        print(rows[-1], flush=True)
    write_csv(os.path.join(a.results_dir, "part1_labl_results.csv"), rows, LABL_COLUMNS)
    return rows


if __name__ == "__main__":
    main()
