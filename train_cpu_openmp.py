#!/usr/bin/env python3
"""CPU thread-scaling benchmark of the native conv1d kernel (reference Module_2/train_cpu_openmp.py):
threads {1,2,4,8,16} x batch {64..512} at K=32, L=500 -> results/part2_openmp_simd_results.csv."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.module2 import run_thread_scaling  # noqa: E402

if __name__ == "__main__":
    for r in run_thread_scaling():
        print(r)
