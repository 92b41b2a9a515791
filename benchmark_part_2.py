#!/usr/bin/env python3
"""Module-2 benchmark (reference Module_2/benchmark_part_2.py): hand-written conv1d vs torch.nn.Conv1d over
B in {64,128,256,512} x K in {3,5,7}, L=500, 15 trials.  On a GPU box: HIP kernel vs MIOpen
(results/part2_hip_results.csv); always: C++ OpenMP/AVX kernel vs CPU torch (results/part2_openmp_results.csv).
Flags: --no-gpu --no-cpu --trials N --plots"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.module2 import (run_part2, time_once, BATCH_SIZES, KERNEL_SIZES, L, TRIALS,  # noqa: E402,F401
                                          WARMUP_STEPS, run_gpu_batch_scaling)
from crossscale_ecg.ops.conv1d import run_omp_conv  # noqa: E402,F401

from crossscale_ecg.utils import usable_cpus  # noqa: E402

NTHREADS = usable_cpus()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-gpu", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--trials", type=int, default=TRIALS)
    ap.add_argument("--threads", type=int, default=NTHREADS)
    ap.add_argument("--results-dir", default="results")
    ap.add_argument("--batch-scaling", action="store_true", help="also sweep GPU batch 64..65536")
    ap.add_argument("--plots", action="store_true")
    a = ap.parse_args(argv)
    out = run_part2(a.results_dir, gpu=not a.no_gpu, cpu=not a.no_cpu, trials=a.trials, nthreads=a.threads)
    if a.batch_scaling and not a.no_gpu:
        run_gpu_batch_scaling(a.results_dir)
    if a.plots:
        from crossscale_ecg.report.plots import plot_part2
        plot_part2(a.results_dir)
    return out


if __name__ == "__main__":
    main()
