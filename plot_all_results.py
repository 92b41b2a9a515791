#!/usr/bin/env python3
"""Reference-compatible entry point (Module_1/plot_all_results.py): merge the A0-A3 and A4 (LABL) CSVs into
``part1_all_results.csv`` with the amortised shard-preparation columns, then draw the throughput comparison
(A0-A4 + effective A4) and the time breakdown at one batch size.

    python plot_all_results.py [--results-dir results] [--batch 512]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.report import plots  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--results-dir", default="results")
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args(argv)
    if not os.path.exists(os.path.join(a.results_dir, "part1_locality_results.csv")):
        raise SystemExit(f"no part1_locality_results.csv in {a.results_dir}")
    outs = plots.plot_all_results_figures(a.results_dir, batch=a.batch)
    print("[csv]", os.path.join(a.results_dir, "part1_all_results.csv"))
    for p in outs:
        print("[plot]", p)


if __name__ == "__main__":
    main()
