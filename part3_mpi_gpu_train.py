#!/usr/bin/env python3
"""Pseudo-federated per-rank training benchmark (API/CLI-compatible with the reference
Module_3/part3_mpi_gpu_train.py).

    torchrun --standalone --nproc-per-node 2 part3_mpi_gpu_train.py --batch-size 256 --steps 200 \
        --data-root data/shards
    mpiexec -n 2 python part3_mpi_gpu_train.py ...     (launcher env shim, no mpi4py needed)

Runs G0 (fp32 baseline), G1 (AMP + side-stream lookahead) and, on a GPU, G0 and G1 on the fused HIP step
(``G0_fused_hip_fp32``: exact fp32 MFMA; ``G1_fused_hip_graph``: bf16); with
``--loader stream`` also the pinned-DataLoader + H2D-stream double-buffer configuration.  Rank 0 appends
BenchStats rows to ``results/part3_mpi_cuda_results.csv`` and prints per-config means over ranks.
"""
from __future__ import annotations

import argparse
import os
import sys
from dataclasses import asdict
from glob import glob

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.config import PseudoFLConfig, add_dataclass_args, from_args  # noqa: E402
from crossscale_ecg.data.dataset import load_shards_to_gpu, make_gpu_batch_iter, make_dataloader  # noqa: E402
from crossscale_ecg.data.shards import assign_shards_evenly, get_shards_for_rank  # noqa: E402,F401
from crossscale_ecg.models.tiny_ecg import TinyECG  # noqa: E402
from crossscale_ecg.parallel.env import init_distributed, shutdown_distributed, setup_device, barrier  # noqa: E402,F401
from crossscale_ecg.parallel.fedavg import Communicator, mpi_avg  # noqa: E402,F401
from crossscale_ecg.train.pseudo_fl import (run_baseline_gpu, run_overlap_gpu, run_fused_gpu,  # noqa: E402
                                            run_stream_overlap)
from crossscale_ecg.utils.csvio import BenchStats, append_results, BENCH_COLUMNS  # noqa: E402,F401


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    add_dataclass_args(ap, PseudoFLConfig)
    cfg = from_args(PseudoFLConfig, ap.parse_args(argv))
    ctx = init_distributed()
    comm = Communicator(ctx)
    dev = ctx.device
    try:
        if cfg.synthetic_windows > 0 or not cfg.data_root:
            n = cfg.synthetic_windows or cfg.max_windows
            g = torch.Generator(device=dev)
            g.manual_seed(1337 + ctx.rank)
            x_gpu = torch.randn((n, cfg.win_len), generator=g, device=dev)
            y_gpu = torch.zeros(n, dtype=torch.long, device=dev)
            local_shards = []
        else:
            all_shards = sorted(glob(os.path.join(cfg.data_root, "ecg_*.bin")))
            if not all_shards:
                raise RuntimeError(f"No shards found in {cfg.data_root}")
            local_shards = assign_shards_evenly(all_shards, ctx.world_size, ctx.rank)
            x_gpu, y_gpu = load_shards_to_gpu(local_shards, dev, max_windows=cfg.max_windows)
        comm.Barrier()
        if x_gpu.size(0) < cfg.batch_size:
            raise RuntimeError("Not enough windows for a single batch on this rank.")
        if ctx.rank == 0 and not cfg.quiet:
            print(f"[pseudo-FL] world={ctx.world_size} device={dev} windows/rank={x_gpu.size(0)}", flush=True)
        log_every = 0 if cfg.quiet else 10
        torch.manual_seed(cfg.seed)
        rows = [asdict(run_baseline_gpu(TinyECG(), make_gpu_batch_iter(x_gpu, y_gpu, cfg.batch_size), dev,
                                        cfg.steps, ctx.rank, cfg.batch_size, log_every=log_every))]
        if dev.type == "cuda":
            amp = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(cfg.amp_dtype, torch.bfloat16)
            torch.manual_seed(cfg.seed)
            rows.append(asdict(run_overlap_gpu(TinyECG(), make_gpu_batch_iter(x_gpu, y_gpu, cfg.batch_size), dev,
                                               cfg.steps, ctx.rank, cfg.batch_size, amp_dtype=amp,
                                               log_every=log_every)))
            if cfg.kernel_backend in ("auto", "fused"):
                for prec in ("fp32", "bf16"):  # native G0 (exact fp32 MFMA) and native G1 (bf16)
                    torch.manual_seed(cfg.seed)
                    rows.append(asdict(run_fused_gpu(TinyECG().to(dev), x_gpu, y_gpu, dev, cfg.steps, ctx.rank,
                                                     cfg.batch_size, seed=cfg.seed + ctx.rank, precision=prec)))
            if cfg.loader == "stream" and local_shards:
                dl, _ = make_dataloader(local_shards, cfg.batch_size, cfg.max_windows, num_workers=2,
                                        pin_memory=True)
                rows.append(asdict(run_stream_overlap(TinyECG(), dl, dev, cfg.steps, ctx.rank, cfg.batch_size)))
        elif ctx.rank == 0:
            print("[WARN] no GPU; skipping the overlap configurations")
        gathered = comm.gather(rows, root=0)
        if ctx.rank == 0:
            flat = [r for per in gathered for r in per]
            append_results(flat, cfg.results_csv, BENCH_COLUMNS)
            print(f"[OK] Appended {len(flat)} rows to {cfg.results_csv}")
            for name in dict.fromkeys(r["config"] for r in flat):
                grp = [r for r in flat if r["config"] == name]
                m = lambda k: sum(r[k] for r in grp) / len(grp)  # noqa: E731
                print(f"=== {name} (mean over {ctx.world_size} ranks): step_ms {m('step_ms'):.4f} "
                      f"data_ms {m('data_ms'):.4f} h2d_ms {m('h2d_ms'):.4f} compute_ms {m('compute_ms'):.4f} "
                      f"samples/s {m('samples_per_s'):,.1f}")
        return rows
    finally:
        shutdown_distributed()


if __name__ == "__main__":
    main()
