"""``shard_prep`` CLI: build ECG shards + ``results/shard_prep_metrics.json``.

Reference: Module_1/shard_prep.py:39-94 (same flags, file names and JSON keys). Fixes the reference
defect that the metrics JSON was written at module level (shard_prep.py:78-94). The synthetic default
count (200,000 windows) matches shard_prep.py:53; ``--n-windows`` overrides it.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import List, Optional

from .shards import make_mitbih_windows, make_synth_windows, write_shard, shard_name


def run_prep(dataset: str = "synthetic", win_len: int = 500, stride: int = 250, shard_size: int = 32768,
             out_dir: str = "data/shards", results_dir: str = "results", n_windows: int = 200000,
             seed: int = 1337, verbose: bool = True) -> dict:
    start = time.perf_counter()
    if dataset == "mitbih":
        windows = make_mitbih_windows(win_len=win_len, stride=stride)
    elif dataset == "synthetic":
        windows = make_synth_windows(N=n_windows, L=win_len, seed=seed)
    else:
        raise ValueError(f"unknown dataset {dataset!r}")
    load_end = time.perf_counter()
    n, l = windows.shape
    if verbose:
        print(f"shard_prep: {n} windows of {l} samples to split")
    os.makedirs(out_dir, exist_ok=True)
    i = sid = 0
    while i < n:
        j = min(i + shard_size, n)
        out = os.path.join(out_dir, shard_name(sid))
        write_shard(out, windows[i:j])
        if verbose:
            print(f"shard_prep: shard {sid}: {j - i} windows -> {out}")
        i, sid = j, sid + 1
    end = time.perf_counter()
    metrics = {
        "dataset": dataset,
        "total_windows": int(n),
        "window_len": int(l),
        "shard_size_windows": int(shard_size),
        "num_shards": int(sid),
        "load_time_s": float(load_end - start),
        "write_time_s": float(end - load_end),
        "total_time_s": float(end - start),
        "timestamp": time.strftime("%Y-%m-%d %H:%M:%S"),
    }
    os.makedirs(results_dir, exist_ok=True)
    with open(os.path.join(results_dir, "shard_prep_metrics.json"), "w") as f:
        json.dump(metrics, f, indent=2)
    if verbose:
        print(f"shard_prep: finished, {sid} shards in {out_dir}; load {metrics['load_time_s']:.2f}s "
              f"write {metrics['write_time_s']:.2f}s; metrics -> {results_dir}/shard_prep_metrics.json")
    return metrics


def main(argv: Optional[List[str]] = None) -> dict:
    ap = argparse.ArgumentParser(description="Write ECG windows as ecg_%05d.bin shards")
    ap.add_argument("--dataset", choices=["mitbih", "synthetic"], default="synthetic")
    ap.add_argument("--win_len", type=int, default=500)
    ap.add_argument("--stride", type=int, default=250)
    ap.add_argument("--shard_size", type=int, default=32768, help="windows per shard")
    ap.add_argument("--n-windows", type=int, default=200000, help="synthetic window count")
    ap.add_argument("--out-dir", default="data/shards")
    ap.add_argument("--results-dir", default="results")
    ap.add_argument("--seed", type=int, default=1337)
    a = ap.parse_args(argv)
    return run_prep(a.dataset, a.win_len, a.stride, a.shard_size, a.out_dir, a.results_dir, a.n_windows, a.seed)


if __name__ == "__main__":
    main()
