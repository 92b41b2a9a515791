"""Federated averaging driver: one FL client per GPU (or per CPU process under gloo).

Reference: TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:137-239 (``main``).  Per configuration (G0 fp32,
G1 AMP) a fresh TinyECG + SGD(lr 1e-2, momentum 0.9); per round: broadcast the global model, run
``local_steps`` local SGD steps on this client's GPU-resident shard, average the weights over clients.
Every round emits a ``RoundStats`` row with the reference's columns (``samples_per_s = n / local_ms``,
excluding comm) and MI355X columns (``comm_exposed_ms``, ``round_wall_ms``); rank 0 appends all rows to
the results CSV and prints node-aggregate samples/s (sum over clients, wall time including comm).

MI355X execution (vs the reference's host-staged per-tensor MPI calls and per-step sync):
  * G1 local round = ONE native hipGraph replay of ``local_steps`` fused HIP steps (``ops.fused_tiny``);
  * FedAvg = ONE RCCL ``all_reduce(AVG)`` of the flat fp32 weight buffer; broadcast = ONE RCCL broadcast;
  * collectives run from a dedicated comm stream with hipEvents on both streams (``parallel.overlap``), so each
    row's ``comm_ms`` is the collectives' own span and ``comm_exposed_ms`` the MEASURED compute-stream stall;
  * ``--overlap tail`` (exact FedAvg): TinyECG / eager clients issue the all-reduce asynchronously and prepare
    the next round's batches before the compute stream waits; the ResNet engine applies the last step's SGD per
    backward segment and all-reduces each segment while earlier segments still run backward;
  * ``--overlap delayed``: the all-reduce runs under the next round's local steps (stale-by-one FedAvg);
  * ResNet1D G1 runs on the native step engine (``train.resnet_trainer``; one hipGraph replay per step);
  * ``--sync none``: pseudo-federated independent clients; ``--sync ddp``: synchronous gradient DP;
  * ``--drop-prob``: client dropout with sample-weighted averaging; ``--ckpt-every``/``--resume``.
"""
from __future__ import annotations

import os
import random
import time
from dataclasses import asdict
from glob import glob
from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import FedAvgConfig
from ..data.dataset import load_shards_to_gpu
from ..data.shards import assign_shards_evenly
from ..models import build_model
from ..parallel.env import DistContext, barrier
from ..parallel.fedavg import Communicator, broadcast_model, weighted_fedavg_, model_flat
from ..parallel.overlap import CommRecord, FedAvgComm, FedAvgRound
from ..utils import profiling, usable_cpus
from ..utils.ckpt import (ckpt_path, save_checkpoint, load_checkpoint, latest_checkpoint, rank_state_path,
                          save_rank_state, load_trainer_local_state)
from ..utils.csvio import RoundStats, append_results, ROUND_COLUMNS
from ..utils.log import RankLogger
from .local import TorchLocalTrainer


def set_basic_seeds(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def _sync(dev: torch.device):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def load_client_data(cfg: FedAvgConfig, ctx: DistContext):
    """This client's windows on its device: shards (round-robin) or on-device synthetic data."""
    dev = ctx.device
    if cfg.synthetic_windows > 0 or not cfg.data_root:
        n = cfg.synthetic_windows if cfg.synthetic_windows > 0 else cfg.max_windows
        n = min(n, cfg.max_windows) if cfg.max_windows else n
        g = torch.Generator(device=dev)
        g.manual_seed(1337 + ctx.rank)
        x = torch.randn((n, cfg.win_len), generator=g, device=dev)
        if cfg.labels == "parity":
            y = (x.mean(1) > 0).long()
        else:
            y = torch.zeros(n, dtype=torch.long, device=dev)
        return x, y
    paths = sorted(glob(os.path.join(cfg.data_root, "ecg_*.bin")))
    if not paths:
        raise RuntimeError(f"No ecg_*.bin files found in {cfg.data_root}")
    mine = assign_shards_evenly(paths, ctx.world_size, ctx.rank)
    return load_shards_to_gpu(mine, dev, max_windows=cfg.max_windows, labels=cfg.labels)


def _amp(cfg: FedAvgConfig):
    return {"bf16": torch.bfloat16, "fp16": torch.float16, "none": None}[cfg.amp_dtype]


def make_trainer(cfg: FedAvgConfig, config_name: str, model, x, y, ctx: DistContext, backend: str):
    seed = cfg.seed + 7919 * ctx.rank
    if backend == "fused":
        from ..ops.fused_tiny import FusedTinyTrainer
        prec = "bf16" if (config_name == "G1" and cfg.amp_dtype == "bf16") else "fp32"
        return FusedTinyTrainer(model, x, y, cfg.batch_size, cfg.local_steps, lr=cfg.lr, momentum=cfg.momentum,
                                seed=seed, precision=prec)
    if backend == "hip":  # ResNet1D on the native step engine
        from .resnet_trainer import ResNetEngineTrainer
        return ResNetEngineTrainer(model, x, y, cfg.batch_size, cfg.local_steps, lr=cfg.lr, momentum=cfg.momentum,
                                   seed=seed, ctx=ctx, sync=cfg.sync, bucket_mb=cfg.bucket_mb)
    amp = None if config_name == "G0" else _amp(cfg)
    net = model
    if cfg.sync == "ddp" and ctx.distributed:
        from torch.nn.parallel import DistributedDataParallel as DDP
        net = DDP(model, device_ids=[dev_index(ctx)] if ctx.device.type == "cuda" else None, bucket_cap_mb=cfg.bucket_mb)
    return TorchLocalTrainer(net, x, y, cfg.batch_size, lr=cfg.lr, momentum=cfg.momentum, amp_dtype=amp, seed=seed)


def dev_index(ctx):
    return ctx.device.index if ctx.device.index is not None else 0


def pick_backend(cfg: FedAvgConfig, config_name: str, ctx: DistContext) -> str:
    if cfg.kernel_backend == "torch" or ctx.device.type != "cuda":
        return "torch"
    if cfg.model.startswith("resnet"):
        if cfg.kernel_backend == "fused":
            raise ValueError("the fused HIP step implements TinyECG only; use --kernel-backend hip for ResNet1D")
        # the MFMA conv kernels compute in bf16: G1 with bf16 AMP only; G0 keeps fp32 semantics on MIOpen
        return "hip" if (config_name == "G1" and cfg.amp_dtype == "bf16") else "torch"
    # fused HIP step: TinyECG in fp32 (G0, or G1 with --amp-dtype none) or bf16 AMP (G1); fp16 AMP keeps the
    # reference's GradScaler path on eager PyTorch
    fused_ok = cfg.model == "tiny_ecg" and (config_name == "G0" or cfg.amp_dtype in ("bf16", "none"))
    if cfg.kernel_backend == "fused":
        if not fused_ok:
            raise ValueError("the fused HIP step implements TinyECG in fp32 or bf16 (not --amp-dtype fp16)")
        return "fused"
    return "fused" if fused_ok else "torch"


def _ddp_fused_round(trainer, ctx: DistContext, n: int):
    """Synchronous data parallel on the fused kernels: grads -> RCCL all-reduce(AVG) -> flat SGD per step."""
    from ..ops import _lib
    from ..ops.fused_tiny import tiny_step_grads
    from ..ops.sgd import FlatSGD
    from ..parallel.fedavg import allreduce_mean_
    if not hasattr(trainer, "_ddp_opt"):
        trainer._ddp_grad = torch.zeros_like(trainer.params)
        trainer._ddp_opt = FlatSGD(trainer.params, trainer._ddp_grad, lr=trainer.lr, momentum=trainer.momentum)
    trainer._loss_steps = n  # batches already drawn by trainer.prepare_round(n) into the staging table
    trainer.idx_table[:n].copy_(trainer.idx_stage[:n])
    trainer._staged = None
    lib = _lib.kernels()
    for s in range(n):
        tiny_step_grads(trainer.params, trainer.x, trainer.y32, trainer.idx_table[s], trainer.B, trainer.nc,
                        trainer.slab, precision=trainer.precision, prefrag=getattr(trainer, "prefrag", None),
                        wprep=getattr(trainer, "wprep", None))
        st = lib.ecg_slab_reduce_sgd(trainer.slab.data_ptr(), trainer.B, trainer.stride, trainer.P, None, None,
                                     trainer._ddp_grad.data_ptr(), trainer.loss_acc.data_ptr(), 0.0, 0.0, 0.0, 0, 0,
                                     None, _lib.stream_ptr(trainer.device))
        _lib.check(st, "ecg_slab_reduce_sgd")
        allreduce_mean_(trainer._ddp_grad, ctx)
        trainer._ddp_opt.step()


def _resume(cfg: FedAvgConfig, cname: str, ctx: DistContext, comm: Communicator, model, trainer, log) -> int:
    """Rank 0 resolves and loads the latest checkpoint and tells every rank the round to start from; each rank
    restores its own client state (momentum, sampler, RNG) when its directory has it (utils/ckpt.py)."""
    path = latest_checkpoint(cfg.ckpt_dir, cname) if ctx.rank == 0 else None
    rnd = -1
    if path:
        st = load_checkpoint(path)
        model.load_state_dict(st["model"])
        rnd = int(st["round"])
    rnd = int(comm.bcast(rnd, root=0))
    if rnd < 0:
        return 0
    own = rank_state_path(cfg.ckpt_dir, rnd, cname, ctx.rank)
    independent = cfg.sync not in ("fedavg", "ddp") or not ctx.distributed
    if os.path.exists(own):
        st = load_checkpoint(own)
        load_trainer_local_state(trainer, st)
        if st.get("client_weights") is not None:  # --sync none: every client continues from its OWN weights
            flat = model_flat(model)
            if st["client_weights"].shape != flat.shape:
                raise ValueError(f"client weights {tuple(st['client_weights'].shape)} != {tuple(flat.shape)}")
            with torch.no_grad():
                flat.copy_(st["client_weights"].to(flat.device))
        elif independent and ctx.rank != 0:
            raise RuntimeError(f"{own} holds no client weights: cannot resume an independent (--sync "
                               f"{cfg.sync}) client without them")
        log.info(f"[fedavg] rank {ctx.rank}: client state restored from {own}")
    elif independent and ctx.rank != 0:
        raise RuntimeError(f"--resume with --sync {cfg.sync}: {own} is missing; an independent client cannot be "
                           "restored from rank 0's model")
    else:
        log.info(f"[fedavg] rank {ctx.rank}: no {own}; momentum restarts at zero, sampler from its seed")
    if ctx.rank == 0:
        log.info(f"[fedavg] resumed {cname} from {path} at round {rnd + 1}")
    return rnd + 1


def run_fedavg(cfg: FedAvgConfig, ctx: DistContext) -> List[Dict]:
    log = RankLogger(ctx.rank, cfg.jsonl, cfg.quiet)
    if "{rank}" in (cfg.ckpt_dir or ""):  # node-local checkpoint directories (no shared filesystem)
        cfg.ckpt_dir = cfg.ckpt_dir.format(rank=ctx.rank)
    comm = Communicator(ctx)
    dev = ctx.device
    torch.set_num_threads(max(1, min(4, usable_cpus())))
    x, y = load_client_data(cfg, ctx)
    if x.shape[0] < cfg.batch_size:
        raise RuntimeError(f"client {ctx.rank} has {x.shape[0]} windows < batch {cfg.batch_size}")
    log.info(f"[fedavg] world={ctx.world_size} backend={ctx.backend} device={dev} windows/client={x.shape[0]} "
             f"L={x.shape[1]} B={cfg.batch_size} rounds={cfg.rounds}x{cfg.local_steps} sync={cfg.sync} "
             f"overlap={cfg.overlap}")
    configs = ["G0", "G1"] if cfg.config == "both" else [cfg.config]
    all_rows: List[Dict] = []
    fcomm = FedAvgComm(ctx)
    for cname in configs:
        set_basic_seeds(cfg.seed + ctx.rank)
        torch.manual_seed(cfg.seed)  # identical init on every client (the round-0 broadcast makes it exact)
        model = build_model(cfg.model, cfg.num_classes).to(dev)
        backend = pick_backend(cfg, cname, ctx)
        if hasattr(model, "flatten_parameters"):
            model.flatten_parameters()
        trainer = make_trainer(cfg, cname, model, x, y, ctx, backend)
        log.info(f"[fedavg] {cname}: kernel backend {backend}")
        start_round = _resume(cfg, cname, ctx, comm, model, trainer, log) if cfg.resume else 0
        fedavg = cfg.sync == "fedavg" and ctx.distributed
        weighted = fedavg and cfg.drop_prob > 0
        mode = cfg.overlap if (fedavg and not weighted) else "none"
        # ResNet engine: the tail step applies SGD per backward segment and all-reduces each segment at once
        seg_tail = mode == "tail" and hasattr(trainer, "tail_fedavg")
        fround = FedAvgRound(model_flat(model), fcomm, "none" if seg_tail else mode)
        if hasattr(trainer, "prepare"):  # capture + upload + warm the round graphs outside round 0's timing
            trainer.prepare([cfg.local_steps - 1 if seg_tail else cfg.local_steps])
        recs = []
        for r in range(start_round, cfg.rounds):
            t_round0 = time.perf_counter()
            rec = CommRecord()
            # ---- broadcast the global model (round 0 / resume / every round for reference parity) ----------
            # (--overlap tail / delayed skip the per-round re-broadcast: it would drain the in-flight all-reduce
            # and serialise the overlap away, and the RCCL AVG already leaves identical weights on every client)
            if ctx.distributed and cfg.sync in ("fedavg", "ddp") and (
                    r == start_round or (fedavg and cfg.bcast_every_round and mode == "none")):
                fround.finalize()  # nothing is in flight here except at a resume boundary
                with profiling.range("bcast"):
                    fcomm.blocking(lambda: broadcast_model(comm, model), rec)
            # ---- local steps (the previous round's tail all-reduce overlaps this round's batch preparation) --
            n = cfg.local_steps - 1 if seg_tail else cfg.local_steps
            m_l0 = fcomm.mark()
            stalls0 = len(fround._rec.stalls) if fround._rec is not None else 0
            prev_rec = fround._rec

            def prep(n=n):
                trainer.prepare_round(n)
                if cfg.inject_prep_delay_ms > 0:  # latency injection (weight-independent host work)
                    time.sleep(cfg.inject_prep_delay_ms / 1e3)

            with profiling.range("local_round"):
                fround.begin_round(prep=prep)
                if cfg.sync == "ddp" and backend == "fused" and ctx.distributed:
                    _ddp_fused_round(trainer, ctx, n)
                else:
                    trainer.launch_round(n)
                if seg_tail:  # the round's last step, its segment all-reduces overlapping its own backward
                    trainer.tail_fedavg(fcomm, rec)
            m_l1 = fcomm.mark()
            # the stall on the previous round's collective happened inside [m_l0, m_l1]: not local work
            inner = prev_rec.stalls[stalls0:] if prev_rec is not None else []
            inner = inner + (rec.stalls if seg_tail else [])
            # ---- FedAvg ----------------------------------------------------------------------------------
            if fedavg:
                with profiling.range("fedavg"):
                    if weighted:
                        rng = random.Random(cfg.seed * 1000003 + r * 8191 + ctx.rank)
                        w = 0.0 if rng.random() < cfg.drop_prob else float(cfg.batch_size * cfg.local_steps)
                        fcomm.blocking(lambda: weighted_fedavg_(model_flat(model), w, ctx), rec)
                    elif not seg_tail:
                        fround.end_round(rec)
            due = bool(cfg.ckpt_every) and (r + 1) % cfg.ckpt_every == 0
            if due and mode != "delayed":
                fround.finalize()  # checkpoints hold averaged weights (drains an in-flight tail all-reduce)
            avg_loss = trainer.avg_loss()
            if due:
                own = model_flat(model) if cfg.sync not in ("fedavg", "ddp") else None  # independent clients
                if ctx.rank == 0:
                    mom = getattr(trainer, "mom", None)
                    with fround.averaged_in_place():  # delayed: avg_r saved, the stale correction stays pending
                        save_checkpoint(ckpt_path(cfg.ckpt_dir, r, cname), r, model, mom, cname, asdict(cfg))
                save_rank_state(cfg.ckpt_dir, r, cname, ctx.rank, trainer, client_weights=own)
            recs.append((r, rec, m_l0, m_l1, inner, avg_loss, (time.perf_counter() - t_round0) * 1e3))
        fround.finalize()
        _sync(dev)
        rows = []
        for r, rec, m_l0, m_l1, inner, avg_loss, wall_ms in recs:
            local_ms = m_l0.ms_to(m_l1) - sum(a.ms_to(b) for a, b in inner)
            row = RoundStats(config=cname, world_size=ctx.world_size, rank=ctx.rank, round_idx=r,
                             batch_size=cfg.batch_size, local_steps=cfg.local_steps, local_train_ms=local_ms,
                             comm_ms=rec.comm_ms(), samples_per_s=cfg.batch_size * cfg.local_steps / (local_ms / 1e3),
                             avg_loss=avg_loss, comm_exposed_ms=rec.exposed_ms(), round_wall_ms=wall_ms,
                             backend=backend, overlap=(cfg.overlap if not weighted else "none")
                             if cfg.sync == "fedavg" else cfg.sync)
            rows.append(asdict(row))
            log.event("round", **asdict(row))
        if hasattr(trainer, "close"):
            trainer.close()
        gathered = comm.gather(rows, root=0)
        if ctx.rank == 0:
            flat_rows = [row for rl in gathered for row in rl]
            all_rows.extend(flat_rows)
            if cfg.results_csv:
                append_results(flat_rows, cfg.results_csv, ROUND_COLUMNS)
            summarize(flat_rows, cname, ctx.world_size, log)
        barrier(ctx)
    return all_rows


def summarize(rows: List[Dict], cname: str, world: int, log: RankLogger) -> Dict[str, float]:
    if not rows:
        return {}
    rounds = sorted({r["round_idx"] for r in rows})
    per_rank = float(np.mean([r["samples_per_s"] for r in rows]))
    node = 0.0
    for ri in rounds:
        rr = [r for r in rows if r["round_idx"] == ri]
        wall = max(r["round_wall_ms"] for r in rr) / 1e3
        node += sum(r["batch_size"] * r["local_steps"] for r in rr) / wall
    node /= len(rounds)
    comm = float(np.mean([r["comm_ms"] for r in rows]))
    local = float(np.mean([r["local_train_ms"] for r in rows]))
    log.info(f"=== {cname} world={world}: per-rank samples/s (ref metric, excl. comm) {per_rank:,.0f} | "
             f"node samples/s (incl. comm) {node:,.0f} | local_ms {local:.3f} comm_ms {comm:.3f} | "
             f"final loss {rows[-1]['avg_loss']:.4f}")
    return {"per_rank_sps": per_rank, "node_sps": node, "comm_ms": comm, "local_ms": local}
