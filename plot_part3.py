#!/usr/bin/env python3
"""Reference-compatible entry point for BOTH Module-3 plot scripts: Module_3/plot_part3.py (pseudo-FL:
throughput vs world size and the grouped h2d + compute breakdown, from ``part3_mpi_cuda_results.csv``) and
Module_3/TRUE_FL_M3/plot_part3.py (FedAvg: per-rank and node throughput vs world size and the local-train / comm
breakdown, from ``fedavg_results_*.csv``).  Draws whichever inputs exist (``--only`` picks one).

    python plot_part3.py [--results-dir results] [--only pseudo|fedavg]
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
    ap.add_argument("--only", choices=["pseudo", "fedavg"], default=None)
    a = ap.parse_args(argv)
    d = a.results_dir
    outs = []
    p3 = os.path.join(d, "part3_mpi_cuda_results.csv")
    if a.only in (None, "pseudo") and os.path.exists(p3):
        outs += plots.plot_pseudo_fl(p3, d)
    if a.only in (None, "fedavg"):
        try:
            outs += plots.plot_fedavg(os.path.join(d, "fedavg_results_*.csv"), d)
        except FileNotFoundError:
            pass
    if not outs:
        raise SystemExit(f"no Module-3 result CSV in {d}")
    for p in outs:
        print("[plot]", p)


if __name__ == "__main__":
    main()
