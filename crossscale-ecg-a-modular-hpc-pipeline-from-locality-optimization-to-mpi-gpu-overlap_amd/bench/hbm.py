"""HBM-scale GPU-resident shards: write multi-GB shard sets, upload them through the native pinned pipeline,
verify them, and train a fused round from the resident data (BASELINE config 5: "288 GB HBM-sized shards").

Reference: ``load_shards_to_gpu`` (Module_3/shard_dataset.py:103-115) does ONE pageable ``.to(device)`` of the
per-rank array, effectively synchronous, and was only ever used at <= 60 MB.  Here
``ops.native_io.upload_shards`` streams mmap'd shards through three pinned staging buffers (multi-threaded host
copy overlapped with the DMA of the previous chunk).

Data: synthetic windows in the reference shard format (``[int64 N][int64 L][N*L float32]``, data/shards.py).
To write GBs quickly each shard tiles one N(0,1) block of 16 Mi floats, shifted by a per-block constant, so
every block differs; the float64 sum of every shard is recorded while writing (the upload check).

    python -m crossscale_ecg.bench.hbm --gb 16 --dir /tmp/ecg_hbm
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import time
from typing import Dict, List, Tuple

import numpy as np
import torch

BLOCK_FLOATS = 1 << 24  # 64 MiB of float32


def _block(seed: int = 1337) -> np.ndarray:
    return np.random.default_rng(seed).standard_normal(BLOCK_FLOATS, dtype=np.float32)


def write_big_shards(out_dir: str, total_gb: float, win_len: int = 500, shard_gb: float = 1.0,
                     seed: int = 1337) -> Tuple[List[str], List[float]]:
    """Write ``ecg_%05d.bin`` shards totalling ``total_gb`` GiB of window data; returns (paths, expected sums).

    Reuses an existing set written with the same parameters (a ``manifest.json`` records them)."""
    os.makedirs(out_dir, exist_ok=True)
    man = os.path.join(out_dir, "manifest.json")
    key = {"total_gb": total_gb, "win_len": win_len, "shard_gb": shard_gb, "seed": seed}
    if os.path.exists(man):
        with open(man) as f:
            m = json.load(f)
        if m.get("key") == key and all(os.path.exists(p) for p in m["paths"]):
            return m["paths"], m["sums"]
    blk = _block(seed)
    rows_per_shard = int(shard_gb * (1 << 30) // (4 * win_len))
    rows_total = int(total_gb * (1 << 30) // (4 * win_len))
    paths, sums = [], []
    done, k, bi = 0, 0, 0
    while done < rows_total:
        n = min(rows_per_shard, rows_total - done)
        p = os.path.join(out_dir, f"ecg_{k:05d}.bin")
        total = n * win_len
        s = 0.0
        with open(p, "wb") as f:
            f.write(np.array([n, win_len], dtype=np.int64).tobytes())
            left = total
            while left > 0:
                take = min(left, BLOCK_FLOATS)
                c = np.float32((bi % 997) * 1e-3)
                chunk = blk[:take] + c
                f.write(chunk.tobytes())
                s += float(chunk.sum(dtype=np.float64))
                left -= take
                bi += 1
        paths.append(p)
        sums.append(s)
        done += n
        k += 1
    with open(man, "w") as f:
        json.dump({"key": key, "paths": paths, "sums": sums}, f)
    return paths, sums


def device_shard_sums(x: torch.Tensor, rows: List[int]) -> List[float]:
    out, r0 = [], 0
    for n in rows:
        acc = torch.zeros((), dtype=torch.float64, device=x.device)
        for a in range(r0, r0 + n, 1 << 20):
            acc += x[a:min(r0 + n, a + (1 << 20))].double().sum()
        out.append(float(acc))
        r0 += n
    return out


def run(gb: float, out_dir: str, threads: int = 0, train: bool = True, keep: bool = True) -> Dict:
    from ..data.shards import shard_header
    from ..ops import native_io
    dev = torch.device("cuda", torch.cuda.current_device())
    t0 = time.perf_counter()
    paths, sums = write_big_shards(out_dir, gb)
    t_write = time.perf_counter() - t0
    rows = [shard_header(p)[0] for p in paths]
    n_rows, L = sum(rows), shard_header(paths[0])[1]
    nbytes = n_rows * L * 4
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x = native_io.upload_shards(paths, dev, n_rows, L, threads=threads or None)
    torch.cuda.synchronize()
    t_up = time.perf_counter() - t0
    # verification: exact float64 sums per shard + bitwise rows sampled from every shard
    dsum = device_shard_sums(x, rows)
    sum_ok = all(abs(a - b) <= 1e-9 * max(1.0, abs(b)) for a, b in zip(dsum, sums))
    rng = np.random.default_rng(0)
    rows_ok, r0 = True, 0
    for p, n in zip(paths, rows):
        mm = np.memmap(p, dtype=np.float32, mode="r", offset=16, shape=(n, L))
        for r in rng.integers(0, n, 8):
            rows_ok &= bool(torch.equal(x[r0 + int(r)].cpu(), torch.from_numpy(np.array(mm[int(r)]))))
        del mm
        r0 += n
    rec = {"gb_uploaded": nbytes / 2**30, "windows": n_rows, "shards": len(paths), "write_s": round(t_write, 2),
           "upload_s": round(t_up, 3), "upload_GBps": round(nbytes / t_up / 1e9, 2), "checksum_ok": sum_ok,
           "rows_bitwise_ok": rows_ok}
    if train:
        from ..models.tiny_ecg import TinyECG
        from ..ops.fused_tiny import FusedTinyTrainer
        y = torch.zeros(n_rows, dtype=torch.long, device=dev)
        torch.manual_seed(0)
        m = TinyECG().to(dev)
        tr = FusedTinyTrainer(m, x, y, 256, 50, seed=1)
        tr.prepare([50])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.run_round(50)
        loss = tr.avg_loss()
        rec["fused_round_ms"] = round((time.perf_counter() - t0) * 1e3, 3)
        rec["fused_round_loss"] = loss
        rec["fused_round_finite"] = bool(np.isfinite(loss))
        tr.close()
        del y
    del x
    torch.cuda.empty_cache()
    if not keep:
        shutil.rmtree(out_dir, ignore_errors=True)
    return rec


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gb", type=float, default=16.0, help="GiB of window data per GPU")
    ap.add_argument("--dir", default="/tmp/ecg_hbm_shards")
    ap.add_argument("--threads", type=int, default=0, help="host copy threads (0: usable CPUs, at most 8)")
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--cleanup", action="store_true", help="delete the shard files afterwards")
    a = ap.parse_args(argv)
    rec = run(a.gb, a.dir, a.threads, not a.no_train, keep=not a.cleanup)
    print(json.dumps(rec), flush=True)
    return rec


if __name__ == "__main__":
    main()
