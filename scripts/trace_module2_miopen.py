#!/usr/bin/env python3
"""Module 2: which MIOpen kernels / HIP calls does ``torch.nn.Conv1d`` run per (B, K) cell, and why are some cells'
single-call latencies ~2x the others?  

``run``: the Module-2 grid (B in {64,128,256,512} x K in {3,5,7}, L=500, fp32, one channel), every cell warmed by an
untimed pass, then ``TRIALS`` single calls exactly as ``bench/module2.time_once`` times them (3 warm-up calls, sync,
ONE timed call, sync), each timed call inside a roctx range "B<b>K<k>".  Run it under

    rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d <dir> -o t -- \\
        python3 scripts/trace_module2_miopen.py run

``parse <dir>``: per cell, the kernels inside the timed range (name, count, device time), the range's wall time, and
the HIP API calls made inside it (count and host time by name) - a solver switch shows up as different kernel names,
a host-side cost as API time the device trace does not have.
"""
import collections
import csv
import glob
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GRID_B = (64, 128, 256, 512)
GRID_K = (3, 5, 7)
L = 500
TRIALS = 15


def run():
    import torch

    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.utils import profiling

    dev = torch.device("cuda")
    torch.manual_seed(0)
    host = {}
    for B in GRID_B:
        for K in GRID_K:
            x = torch.randn(B, 1, L, device=dev)
            conv = torch.nn.Conv1d(1, 1, K, bias=False).to(dev)
            with torch.no_grad():
                for _ in range(10):  # untimed warm pass of this cell
                    conv(x)
                torch.cuda.synchronize()
                ts = []
                for _ in range(TRIALS):
                    for _ in range(3):
                        conv(x)
                    torch.cuda.synchronize()
                    with profiling.range(f"B{B}K{K}"):
                        t0 = time.perf_counter()
                        conv(x)
                        torch.cuda.synchronize()
                        ts.append((time.perf_counter() - t0) * 1e6)
            host[(B, K)] = statistics.median(ts)
            print(f"B={B} K={K}: time_once median {host[(B, K)]:.1f} us", flush=True)


def _rows(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def _short(name, n=90):
    return name if len(name) <= n else name[:n] + "..."


def parse(d):
    markers = _rows(d, "*marker_api_trace.csv")
    kernels = _rows(d, "*kernel_trace.csv")
    hip = _rows(d, "*hip_api_trace.csv")
    ranges = collections.defaultdict(list)
    for m in markers:
        name = m.get("Function") or m.get("Marker_Name") or ""
        if name.startswith("B") and "K" in name:
            ranges[name].append((int(m["Start_Timestamp"]), int(m["End_Timestamp"])))
    kin = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"]) for k in kernels]
    hin = [(int(h["Start_Timestamp"]), int(h["End_Timestamp"]), h.get("Function", h.get("Operation", "?")))
           for h in hip]
    for B in GRID_B:
        for K in GRID_K:
            key = f"B{B}K{K}"
            rs = ranges.get(key, [])
            if not rs:
                continue
            wall = statistics.median((e - s) / 1e3 for s, e in rs)
            kn, kt, api_n, api_t = collections.Counter(), collections.defaultdict(list), collections.Counter(), \
                collections.defaultdict(float)
            for s, e in rs:
                for ks, ke, name in kin:
                    if s <= ks and ke <= e + 200_000:  # kernels launched in the range (end within 200 us)
                        kn[name] += 1
                        kt[name].append((ke - ks) / 1e3)
                for hs, he, name in hin:
                    if s <= hs and he <= e:
                        api_n[name] += 1
                        api_t[name] += (he - hs) / 1e3
            print(f"== {key}: timed-call wall median {wall:.1f} us over {len(rs)} calls")
            for name, c in kn.most_common():
                print(f"   kernel x{c / len(rs):.1f}/call  {statistics.median(kt[name]):7.2f} us  {_short(name)}")
            for name, c in api_n.most_common(6):
                print(f"   hip    x{c / len(rs):.1f}/call  {api_t[name] / len(rs):7.2f} us/call host  {name}")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "parse":
        parse(sys.argv[2])
    else:
        run()
