"""Result records and CSV writers with the reference's exact column schemas.

* ``BenchStats``  <- Module_3/part3_mpi_gpu_train.py:64-75 (``part3_mpi_cuda_results.csv``)
* ``RoundStats``  <- TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:44-55 (``fedavg_results*.csv``), extended with
  MI355X-only columns appended AFTER the reference ones (``comm_exposed_ms``, ``node_samples_per_s``, ...)
* ``append_results`` <- part3_mpi_gpu_train.py:33-61 (header-aligned append, retry on PermissionError)
* ``safe_write_csv`` <- Module_2/benchmark_part_2.py:111-121 (timestamped fallback when locked)
"""
from __future__ import annotations

import csv
import os
import time
from dataclasses import dataclass, field, fields, asdict
from typing import Dict, Iterable, List, Sequence


@dataclass
class BenchStats:
    config: str
    world_size: int
    rank: int
    batch_size: int
    steps: int
    data_ms: float
    h2d_ms: float
    compute_ms: float
    step_ms: float
    samples_per_s: float


@dataclass
class RoundStats:
    config: str
    world_size: int
    rank: int
    round_idx: int
    batch_size: int
    local_steps: int
    local_train_ms: float
    comm_ms: float
    samples_per_s: float
    avg_loss: float
    # ---- MI355X additions (not in the reference schema) ----
    comm_exposed_ms: float = 0.0
    round_wall_ms: float = 0.0
    backend: str = ""
    overlap: str = ""


BENCH_COLUMNS = [f.name for f in fields(BenchStats)]
ROUND_COLUMNS_REF = ["config", "world_size", "rank", "round_idx", "batch_size", "local_steps", "local_train_ms",
                     "comm_ms", "samples_per_s", "avg_loss"]
ROUND_COLUMNS = [f.name for f in fields(RoundStats)]

LOCALITY_COLUMNS = ["config", "batch_size", "pin_memory", "contiguous", "non_blocking", "data_ms", "h2d_ms",
                    "compute_ms", "step_ms", "samples_per_s"]
LABL_COLUMNS = ["config", "batch_size", "step_ms", "samples_per_s", "data_ms", "h2d_ms", "compute_ms"]
PART2_COLUMNS = ["batch_size", "kernel_size", "nthreads", "torch_ms_median", "torch_ms_mean", "torch_ms_std",
                 "torch_ms_p95", "omp_ms_median", "omp_ms_mean", "omp_ms_std", "omp_ms_p95", "torch_sps", "omp_sps",
                 "speedup_med"]
PART2_RAW_COLUMNS = ["batch_size", "kernel_size", "trial", "torch_ms", "omp_ms"]
PART2_SCALING_COLUMNS = ["threads", "batch", "compute_ms", "samples_per_s"]


def _rows_to_dicts(rows) -> List[Dict]:
    out = []
    for r in rows:
        out.append(asdict(r) if hasattr(r, "__dataclass_fields__") else dict(r))
    return out


def write_csv(path: str, rows, columns: Sequence[str]) -> str:
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(columns), extrasaction="ignore")
        w.writeheader()
        for r in _rows_to_dicts(rows):
            w.writerow(r)
    return path


def safe_write_csv(rows, path: str, columns: Sequence[str]) -> str:
    try:
        return write_csv(path, rows, columns)
    except PermissionError:
        base, ext = os.path.splitext(path)
        fb = f"{base}_{int(time.time())}{ext}"
        print(f"[WARN] {os.path.abspath(path)} locked. Wrote {os.path.abspath(fb)}")
        return write_csv(fb, rows, columns)


def read_csv(path: str) -> List[Dict[str, str]]:
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def append_results(rows, path: str, columns: Sequence[str] | None = None, max_retries: int = 20) -> str:
    """Append rows; if the file exists, align to its header (extra columns dropped, missing -> empty)."""
    dicts = _rows_to_dicts(rows)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    for _attempt in range(max_retries):
        try:
            if os.path.exists(path) and os.path.getsize(path) > 0:
                with open(path, newline="") as f:
                    header = next(csv.reader(f))
                with open(path, "a", newline="") as f:
                    w = csv.DictWriter(f, fieldnames=header, extrasaction="ignore")
                    for r in dicts:
                        w.writerow({k: r.get(k, "") for k in header})
            else:
                cols = list(columns) if columns else (list(dicts[0].keys()) if dicts else [])
                write_csv(path, dicts, cols)
            return path
        except PermissionError:
            time.sleep(0.25)
    raise RuntimeError(f"Could not write CSV after {max_retries} attempts: {path}")
