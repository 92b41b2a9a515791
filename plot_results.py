#!/usr/bin/env python3
"""Regenerate every figure from the result CSVs (reference plot_locality.py, plot_all_results.py,
plot_part2.py, plot_part3.py x2).  python plot_results.py [--results-dir results]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.report import plots  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--results-dir", default="results")
    a = ap.parse_args(argv)
    d = a.results_dir
    made = []
    loc = os.path.join(d, "part1_locality_results.csv")
    if os.path.exists(loc):
        made += plots.plot_locality(loc, d)
        made += plots.plot_all_results_figures(d)
    made += plots.plot_part2(d)
    p3 = os.path.join(d, "part3_mpi_cuda_results.csv")
    if os.path.exists(p3):
        made += plots.plot_pseudo_fl(p3, d)
    try:
        made += plots.plot_fedavg(os.path.join(d, "fedavg_results*.csv"), d)
    except FileNotFoundError:
        pass
    for m in made:
        print("[plot]", m)


if __name__ == "__main__":
    main()
