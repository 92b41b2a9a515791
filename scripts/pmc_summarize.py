#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--pmc ... --kernel-trace --output-format csv`` counter collection per kernel.

Achieved bf16 matrix throughput per kernel = SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 FLOP over the kernel's time. Two
times are used: the dispatch durations of the PMC run itself (counter collection serialises dispatches) and, when a
``--stats`` kernel CSV of a run without counters is given, its average duration per kernel.

    python scripts/pmc_summarize.py <counter_collection.csv> [kernel_stats.csv] [top=14] [pass2_counter_collection.csv]

A second pass with SQ_WAVE_CYCLES (and SQ_WAIT_ANY / SQ_ACTIVE_INST_ANY) adds per-wave fractions, which do not grow
with the number of waves per CU as ``SQ_WAIT_INST_LDS / SQ_BUSY_CYCLES`` does: LDS-wait/wave = SQ_WAIT_INST_LDS /
SQ_WAVE_CYCLES (both summed over waves, quad-cycles), matched per kernel name across the two runs.
"""
import collections
import csv
import re
import sys

PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 (no sparsity)


def short(name):
    m = re.search(r"::(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def per_dispatch(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return {k: {c: v / len(disp[k]) for c, v in a.items()} for k, a in agg.items()}


def main(path, stats=None, top=14, pass2=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    dur = {}
    p2 = per_dispatch(pass2) if pass2 else {}
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        dur.setdefault((k, r["Dispatch_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = collections.defaultdict(float)
    for (k, _), v in dur.items():
        tot[k] += v
    avg_ns = {}
    if stats:
        for r in csv.DictReader(open(stats)):
            avg_ns[short(r["Name"])] = float(r["AverageNs"])
    mops = "SQ_INSTS_VALU_MFMA_MOPS_BF16"
    print(f"{'kernel':48s} {'disp':>5s} {'GFLOP/disp':>10s} {'TF/s pmc':>8s} {'TF/s run':>8s} {'%peak':>6s} "
          f"{'LDSconf/idx':>11s} {'LDSwait/busy':>12s}" + (f" {'LDSwait/wave':>12s} {'wait/wave':>9s} {'issue/wave':>10s}"
                                                            if p2 else ""))
    for k in sorted(agg, key=lambda k: -agg[k][mops])[:top]:
        a, n = agg[k], len(disp[k])
        if a[mops] == 0:
            continue
        gf = a[mops] * 512 / n / 1e9
        tf_pmc = a[mops] * 512 / tot[k] / 1e3
        tf_run = gf / avg_ns[k] * 1e6 if k in avg_ns else float("nan")
        print(f"{k[:48]:48s} {n:5d} {gf:10.2f} {tf_pmc:8.0f} {tf_run:8.0f} {100 * tf_run / PEAK_BF16_TFLOPS:6.1f} "
              f"{a['SQ_LDS_BANK_CONFLICT'] / max(1.0, a['SQ_LDS_IDX_ACTIVE']):11.3f} "
              f"{a['SQ_WAIT_INST_LDS'] / max(1.0, a['SQ_BUSY_CYCLES']):12.3f}", end="")
        if p2:
            b = p2.get(k, {})
            wc = b.get("SQ_WAVE_CYCLES", 0.0)
            if wc:
                print(f" {a['SQ_WAIT_INST_LDS'] / n / wc:12.3f} {b.get('SQ_WAIT_ANY', 0.0) / wc:9.3f} "
                      f"{b.get('SQ_ACTIVE_INST_ANY', 0.0) / wc:10.3f}", end="")
        print()


if __name__ == "__main__":
    args = sys.argv[1:]
    main(args[0], args[1] if len(args) > 1 and args[1] else None, int(args[2]) if len(args) > 2 else 14,
         args[3] if len(args) > 3 else None)
