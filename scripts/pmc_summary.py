#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs per kernel family: mean per dispatch of each counter, plus derived
MFMA busy / LDS-wait / bank-conflict fractions when the counters are present.

    python scripts/pmc_summary.py <counter_collection.csv> [...] [--match SUBSTR] [--grid] [--top N]
Kernels are grouped by name with template arguments kept (``--grid`` also splits by grid size).
"""
import argparse
import collections
import csv


def load(paths, match):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                if match and match not in k:
                    continue
                key = (k, r.get("Grid_Size", "")) if GRID else (k, "")
                rows[key][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = {}
    for key, d in rows.items():
        per = collections.defaultdict(list)
        disp = set()
        for (did, cn), vals in d.items():
            per[cn].append(sum(vals))
            disp.add(did)
        out[key] = ({cn: sum(v) / len(v) for cn, v in per.items()}, len(disp))
    return out


def short(name):
    n = name.split("(")[0]
    return n.replace("(anonymous namespace)::", "")[:90]


def main():
    global GRID
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--grid", action="store_true")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    GRID = a.grid
    res = load(a.csv, a.match)
    for (k, g), (c, n) in sorted(res.items(), key=lambda kv: -kv[1][0].get("SQ_BUSY_CYCLES", kv[1][0].get(
            "SQ_WAVE_CYCLES", 0)))[: a.top]:
        line = f"{short(k)}{' grid=' + g if g else ''} n={n}"
        parts = [f"{cn}={v:.4g}" for cn, v in sorted(c.items())]
        der = []
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "SQ_BUSY_CYCLES" in c and c["SQ_BUSY_CYCLES"]:
            der.append(f"mfma_busy/busy={c['SQ_VALU_MFMA_BUSY_CYCLES'] / (c['SQ_BUSY_CYCLES'] * 4 * 32):.3f}")
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            der.append(f"lds_conflict/active={c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "SQ_WAIT_INST_LDS" in c and c.get("SQ_WAVE_CYCLES"):
            der.append(f"wait_lds/wave={c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.3f}")
        for nm in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if nm in c and c.get("SQ_WAVE_CYCLES"):
                der.append(f"{nm[3:].lower()}/wave={c[nm] / c['SQ_WAVE_CYCLES']:.3f}")
        print(line)
        print("   " + " ".join(parts))
        if der:
            print("   " + " ".join(der))


GRID = False
if __name__ == "__main__":
    main()
