#!/usr/bin/env python3
"""Headline benchmark: TinyECG FedAvg training throughput (ECG samples/s, whole node) on MI355X.

Config (BASELINE.json / Module_3/TRUE_FL_M3/run_part3_sweep.sh:38-49): TinyECG (1,458 params),
batch 256 per client, window L=500, <=20,000 windows per client, FedAvg every 50 local steps,
SGD(lr=1e-2, momentum=0.9), AMP (bf16 here), one FL client per GPU (``--gpus N`` ranks over RCCL).

A "step" = one local SGD step of every client (N x 256 samples).  W warmup steps, then exactly K
timed steps bracketed by barrier + synchronize; FedAvg all-reduces every ``--local-steps`` steps inside
the timed region.  Reported value = N * 256 * K / max-over-ranks(elapsed)  (whole-job samples/s).
Data: synthetic N(0,1) windows generated on device (the reference's synthetic shard distribution,
Module_1/shard_prep.py:35-37), dummy zero labels (Module_3/shard_dataset.py:70), random-init weights.

Extra fields: ``torch_eager_*`` (same step in eager PyTorch bf16-autocast, the reference's G1 code path,
measured in the same process) and ``conv1d_*`` (Module-2 kernel vs torch.nn.Conv1d, B=256, K=7).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import crossscale_ecg  # noqa: E402
from crossscale_ecg.models.tiny_ecg import TinyECG, num_params  # noqa: E402
from crossscale_ecg.parallel.env import init_distributed, barrier  # noqa: E402
from crossscale_ecg.parallel.fedavg import allreduce_mean_  # noqa: E402

METRIC = "ECG samples/sec (node) + conv1d speedup vs torch.Conv1d, tiny 1D-CNN at 1/2/4/8 GPU"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--model", choices=["tiny_ecg", "resnet1d34", "resnet1d18"], default="tiny_ecg",
                    help="tiny_ecg = BASELINE headline; resnet1d34 = BASELINE config 5 (scaling stress)")
    ap.add_argument("--batch-size", type=int, default=None, help="per client (default 256; 1024 for ResNet1D)")
    ap.add_argument("--local-steps", type=int, default=50)
    ap.add_argument("--max-windows", type=int, default=20000)
    ap.add_argument("--win-len", type=int, default=500)
    ap.add_argument("--backend", choices=["fused", "torch"], default="fused")
    ap.add_argument("--no-extras", action="store_true", help="skip torch-eager and conv1d side measurements")
    return ap.parse_args(argv)


def timed_fused(trainer, ctx, steps, local_steps, flat):
    done = 0
    since_sync = 0
    while done < steps:
        n = min(local_steps - since_sync, steps - done)
        trainer.run_round(n, reset_loss=False)
        done += n
        since_sync += n
        if since_sync == local_steps:
            allreduce_mean_(flat, ctx)  # FedAvg: one RCCL all-reduce (AVG) of the flat weights
            since_sync = 0
    return done


def torch_eager_rate(x, y, B, steps, device):
    import torch.nn.functional as F
    model = TinyECG().to(device)
    opt = torch.optim.SGD(model.parameters(), lr=1e-2, momentum=0.9)
    g = torch.Generator(device=device)
    g.manual_seed(0)

    def one():
        sel = torch.randint(0, x.shape[0], (B,), device=device, generator=g)
        xb, yb = x[sel].unsqueeze(1), y[sel]
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(model(xb), yb)
        loss.backward()
        opt.step()
        return loss

    for _ in range(10):
        one()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        one()
    torch.cuda.synchronize()
    return B * steps / (time.perf_counter() - t0)


def conv1d_speedup(device, B=256, L=500, K=7, trials=15, inner=20):
    from crossscale_ecg.ops.conv1d import conv1d_valid
    x = torch.randn(B, 1, L, device=device)
    w = torch.randn(K, device=device)
    conv = torch.nn.Conv1d(1, 1, K, bias=False).to(device)
    with torch.no_grad():
        conv.weight.copy_(w.view(1, 1, K))
    out = torch.empty(B, L - K + 1, device=device)

    def t_call(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(inner):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / inner

    with torch.no_grad():
        tt = [t_call(lambda: conv(x)) for _ in range(trials)]
        th = [t_call(lambda: conv1d_valid(x[:, 0], w, backend="hip", out=out)) for _ in range(trials)]
    return statistics.median(tt), statistics.median(th)


def main(argv=None):
    a = parse(argv)
    ctx = init_distributed()
    if ctx.world_size != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={ctx.world_size}; launch with torchrun for N>1")
    dev = ctx.device
    if dev.type != "cuda":
        raise SystemExit("bench.py needs a GPU")
    resnet = a.model.startswith("resnet")
    if a.batch_size is None:
        a.batch_size = 1024 if resnet else 256
    B, S = a.batch_size, a.local_steps
    # per-client synthetic shard, resident in HBM
    gen = torch.Generator(device=dev)
    gen.manual_seed(1337 + ctx.rank)
    x = torch.randn((a.max_windows, a.win_len), generator=gen, device=dev, dtype=torch.float32)
    y = torch.zeros(a.max_windows, dtype=torch.long, device=dev)

    torch.manual_seed(1234)  # same initial global model on every client (== round-0 broadcast)
    if resnet:
        from crossscale_ecg.models import build_model
        model = build_model(a.model, 2).to(dev)
    else:
        model = TinyECG(num_classes=2).to(dev)
    flat = model.flatten_parameters()

    if resnet and a.backend == "fused":  # native ResNet step engine (one hipGraph per step)
        from crossscale_ecg.train.resnet_trainer import ResNetEngineTrainer
        trainer = ResNetEngineTrainer(model, x, y, B, S, lr=1e-2, momentum=0.9, seed=4321 + ctx.rank, ctx=ctx)
        run = lambda k: timed_fused(trainer, ctx, k, S, flat)  # noqa: E731
    elif a.backend == "fused":
        from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
        trainer = FusedTinyTrainer(model, x, y, B, S, lr=1e-2, momentum=0.9, seed=4321 + ctx.rank)
        run = lambda k: timed_fused(trainer, ctx, k, S, flat)  # noqa: E731
    else:
        from crossscale_ecg.train.local import TorchLocalTrainer
        trainer = TorchLocalTrainer(model, x, y, B, amp_dtype=torch.bfloat16, seed=4321 + ctx.rank)

        def run(k):
            done = 0
            while done < k:
                n = min(S, k - done)
                trainer.run_steps(n)
                done += n
                if n == S:
                    allreduce_mean_(flat, ctx)
            return done

    # warmup (also builds the graphs)
    if a.warmup > 0:
        run(a.warmup)
    torch.cuda.synchronize(dev)
    barrier(ctx)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(a.steps)
    torch.cuda.synchronize(dev)
    barrier(ctx)
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if ctx.distributed:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total = a.gpus * B * a.steps
    value = total / elapsed
    loss = trainer.avg_loss() if hasattr(trainer, "avg_loss") else float("nan")

    extras = {}
    if ctx.rank == 0 and not a.no_extras and resnet:
        try:
            from crossscale_ecg.bench.resnet import train_throughput
            extras["torch_eager_samples_per_s_per_gpu"] = round(train_throughput("torch", B=B, L=a.win_len), 1)
            extras["speedup_vs_torch_eager_per_gpu"] = round(value / a.gpus / extras["torch_eager_samples_per_s_per_gpu"], 2)
        except Exception as e:  # pragma: no cover
            extras["torch_eager_error"] = repr(e)[:200]
    elif ctx.rank == 0 and not a.no_extras:
        try:
            extras["torch_eager_samples_per_s_per_gpu"] = round(torch_eager_rate(x, y, B, 100, dev), 1)
            extras["speedup_vs_torch_eager_per_gpu"] = round(value / a.gpus / extras["torch_eager_samples_per_s_per_gpu"], 2)
        except Exception as e:  # pragma: no cover
            extras["torch_eager_error"] = repr(e)[:200]
        try:
            tm, hm = conv1d_speedup(dev)
            extras["conv1d_torch_ms_median"] = round(tm, 5)
            extras["conv1d_hip_ms_median"] = round(hm, 5)
            extras["conv1d_speedup_vs_torch"] = round(tm / hm, 3)
        except Exception as e:  # pragma: no cover
            extras["conv1d_error"] = repr(e)[:200]

    if ctx.rank == 0:
        n_par = sum(p.numel() for p in model.parameters())
        rec = {
            "metric": METRIC if not resnet else "ECG samples/sec (node), ResNet1D-34 scaling-stress config (BASELINE config 5)",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic",
            "config": {
                "model": f"TinyECG ({num_params(2)} params)" if not resnet else f"{a.model} ({n_par} params)",
                "global_batch": B * a.gpus,
                "seq_len": a.win_len,
                "parallelism": f"dp{a.gpus}",
                "sync": f"fedavg every {S} local steps ({'RCCL' if ctx.backend in ('nccl', 'none') else ctx.backend} all_reduce AVG)",
                "per_client_batch": B,
                "max_windows_per_client": a.max_windows,
                "backend": a.backend,
            },
            "final_avg_loss": round(loss, 6) if loss == loss else None,
            **extras,
        }
        print(json.dumps(rec), flush=True)
    if hasattr(trainer, "close"):
        trainer.close()


if __name__ == "__main__":
    main()
