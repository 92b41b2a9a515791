#!/usr/bin/env python3
"""Per-kernel durations and the gaps between consecutive kernels from a rocprofv3 kernel_trace.csv (the
two-launch TinyECG round: step kernel -> slab reduce -> step kernel ...).  Usage: trace_gaps.py trace.csv"""
import csv
import statistics
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    short = lambda n: ("step" if "tiny_ecg_step" in n else "reduce" if "slab_reduce" in n else  # noqa: E731
                       "prep" if "tiny_prep" in n else n[:30])
    dur, gap = {}, {}
    for (n0, s0, e0), (n1, s1, e1) in zip(ks, ks[1:]):
        a, b = short(n0), short(n1)
        dur.setdefault(a, []).append((e0 - s0) / 1e3)
        if a in ("step", "reduce", "prep") and b in ("step", "reduce"):
            gap.setdefault(f"{a}->{b}", []).append((s1 - e0) / 1e3)
    for k, v in dur.items():
        if len(v) > 5:
            print(f"{k:32s} n={len(v):5d} median {statistics.median(v):8.3f} us  p10 {sorted(v)[len(v)//10]:8.3f}  "
                  f"p90 {sorted(v)[9*len(v)//10]:8.3f}")
    for k, v in gap.items():
        print(f"gap {k:28s} n={len(v):5d} median {statistics.median(v):8.3f} us  p10 {sorted(v)[len(v)//10]:8.3f}  "
              f"p90 {sorted(v)[9*len(v)//10]:8.3f}")
    steps = [s for n, s, e in ks if short(n) == "step"]
    d = [(b - a) / 1e3 for a, b in zip(steps, steps[1:])]
    print(f"step-to-step period median {statistics.median(d):.3f} us")


if __name__ == "__main__":
    main(sys.argv[1])
