#!/usr/bin/env python3
"""Reference-compatible entry point (Module_2/plot_part2.py): the Module-2 figures - HIP and C++ OpenMP conv1d
throughput / speedup over torch per kernel width, and the CPU thread-scaling curve.

    python plot_part2.py [--results-dir results]
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
    a = ap.parse_args(argv)
    outs = plots.plot_part2(a.results_dir)
    if not outs:
        raise SystemExit(f"no Module-2 CSV in {a.results_dir}")
    for p in outs:
        print("[plot]", p)


if __name__ == "__main__":
    main()
