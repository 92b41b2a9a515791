#!/usr/bin/env python3
"""Reference-compatible entry point (Module_1/plot_locality.py): the A0-A3(+) locality figures - throughput vs
batch size and the per-step data / h2d / compute breakdown at ``--batch``.

    python plot_locality.py [--results-dir results] [--csv part1_locality_results.csv] [--batch 512]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.report import plots  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description="Plot A0-A3 locality results")
    ap.add_argument("--results-dir", default=None, help="Path to results/ (default: ./results)")
    ap.add_argument("--csv", default="part1_locality_results.csv", help="CSV with the A0-A3 results")
    ap.add_argument("--batch", type=int, default=512, help="batch size of the time-breakdown figure")
    a = ap.parse_args(argv)
    d = a.results_dir or os.path.join(os.getcwd(), "results")
    path = a.csv if os.path.isabs(a.csv) else os.path.join(d, a.csv)
    if not os.path.exists(path):
        raise SystemExit(f"CSV not found: {path}")
    for p in plots.plot_locality(path, d, batch=a.batch):
        print("[plot]", p)


if __name__ == "__main__":
    main()
