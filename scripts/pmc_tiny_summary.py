#!/usr/bin/env python3
"""Per-wave counters of the TinyECG step kernel from a ``rocprofv3 --pmc`` counter CSV (scripts/gpu_session.sh
tinypmc): medians over the dispatches of tiny_ecg_step_kernel<16,0,false,true> of VALU / SALU / LDS instructions per
wave, wave cycles per wave (SQ_WAVE_CYCLES counts 4-cycle quanta: x4) and SQ_WAIT_ANY / SQ_WAVE_CYCLES - the row format of profiles/r5/pmc/tiny_step_pmc.txt.

    python scripts/pmc_tiny_summary.py <p_counter_collection.csv> [label]
"""
import collections
import csv
import statistics
import sys

KERNEL = "tiny_ecg_step_kernel<16, 0, false, true>"


def main(path, label="?"):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if KERNEL not in r["Kernel_Name"]:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    rows = [d for d in per.values() if d.get("SQ_WAVES")]
    med = lambda k: statistics.median(d[k] / d["SQ_WAVES"] for d in rows)  # noqa: E731
    wait = statistics.median(d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"] for d in rows)
    print(f"{label:<9} {'':<38} {med('SQ_INSTS_VALU'):9.1f} {med('SQ_INSTS_SALU'):9.1f} {med('SQ_INSTS_LDS'):8.1f} "
          f"{4 * med('SQ_WAVE_CYCLES'):11.0f} {wait:10.3f}   ({len(rows)} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "?")
