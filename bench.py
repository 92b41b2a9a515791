#!/usr/bin/env python3
"""Headline benchmark: TinyECG FedAvg training throughput (ECG samples/s, whole node) on MI355X.

Config (BASELINE.json / Module_3/TRUE_FL_M3/run_part3_sweep.sh:38-49): TinyECG (1,458 params),
batch 256 per client, window L=500, <=20,000 windows per client, FedAvg every 50 local steps,
SGD(lr=1e-2, momentum=0.9), AMP (bf16 here), one FL client per GPU (``--gpus N`` ranks over RCCL).

A "step" = one local SGD step of every client (N x 256 samples).  The step sequence is cut into FedAvg
rounds of ``--local-steps`` steps; EVERY round - including a trailing partial one - ends with the FedAvg
all-reduce (one RCCL ``all_reduce(AVG)`` of the flat weights, reference part3_fedavg_overlap_mpi_gpu.py:
209-211), so the timed region always contains communication.  W warmup steps (same round plan), then
every hipGraph the timed plan needs is captured and uploaded, then exactly K timed steps bracketed by
barrier (a shared-memory host barrier when all ranks share the node, parallel/host_barrier.py) + synchronize;
value = N * B * K / max-over-ranks(elapsed) (whole-job samples/s).  Each round's
batch indices are drawn while the previous round computes (the first timed round's behind the last warmup
round) and copied into the step table by the round graph's first node.

Launch: ``python bench.py --gpus N`` with N > 1 and no launcher environment starts N ranks itself
(``torch.distributed.run`` as a child process, one rank per GPU); the parent never touches the GPU.
Under torchrun / mpiexec / srun (RANK+WORLD_SIZE set) it runs as one rank.

Data: synthetic N(0,1) windows generated on device (the reference's synthetic shard distribution,
Module_1/shard_prep.py:35-37), dummy zero labels (Module_3/shard_dataset.py:70), random-init weights.

Extra fields: ``torch_eager_*`` (same step in eager PyTorch bf16-autocast, the reference's G1 code path,
measured in the same process) and ``conv1d_*`` (Module-2 kernel vs torch.nn.Conv1d, B=256, K=7; the
headline ``conv1d_speedup_vs_torch`` uses the reference's single-call ``time_once`` metric,
Module_2/benchmark_part_2.py:61-67,108).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
METRIC = "ECG samples/sec (node) + conv1d speedup vs torch.Conv1d, tiny 1D-CNN at 1/2/4/8 GPU"
_LAUNCHER_VARS = ("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "PMIX_SIZE", "SLURM_NTASKS")


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
    ap.add_argument("--overlap", choices=["none", "tail"], default="tail",
                    help="tail: the FedAvg all-reduce of round r runs under round r+1's batch preparation "
                         "(exact FedAvg, bitwise equal to none)")
    ap.add_argument("--device", choices=["gpu", "cpu"], default="gpu",
                    help="cpu: plumbing rehearsal of the launch/sync/JSON contract (gloo, eager torch)")
    ap.add_argument("--no-extras", action="store_true", help="skip torch-eager and conv1d side measurements")
    ap.add_argument("--no-numa-bind", action="store_true",
                    help="keep the inherited CPU affinity (default: each rank pins itself to its GPU's NUMA node)")
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------------- self-launch
def _under_launcher() -> bool:
    return any(v in os.environ for v in _LAUNCHER_VARS)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def count_gpus_kfd(root: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPUs visible to this process, counted WITHOUT the HIP runtime: KFD topology nodes with a non-zero
    ``gpu_id`` (CPU nodes have 0), limited by ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` /
    ``CUDA_VISIBLE_DEVICES`` when set.  -1 when the topology is not readable (no KFD)."""
    try:
        nodes = os.listdir(root)
    except OSError:
        return -1
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(root, node, "gpu_id")) as f:
                n += int(f.read().strip() or 0) != 0
        except (OSError, ValueError):
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([t for t in v.split(",") if t.strip()]))
    return n


def self_launch(a, argv) -> int:
    """Start ``a.gpus`` ranks (one per GPU) as a ``torch.distributed.run`` child; return its exit code.

    The parent never touches the GPU runtime: it neither imports torch nor calls HIP; GPUs are counted from
    the KFD sysfs topology (``count_gpus_kfd``)."""
    backend = os.environ.get("ECG_DIST_BACKEND", "nccl")
    if a.device == "gpu" and backend == "nccl":
        n_dev = count_gpus_kfd()
        if 0 <= n_dev < a.gpus:
            print(f"bench.py: --gpus {a.gpus} needs {a.gpus} GPUs for RCCL (one rank per GPU), found {n_dev}",
                  file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


# ----------------------------------------------------------------------------------- timed loop
def round_plan(steps: int, local_steps: int):
    """Round lengths covering ``steps`` local steps: full rounds, then one trailing partial round."""
    full, rem = divmod(int(steps), int(local_steps))
    return [local_steps] * full + ([rem] if rem else [])


class FedAvgRunner:
    """Runs a round plan on a trainer: each round = local steps then the FedAvg all-reduce (AVG).

    The collectives go through ``parallel.overlap.FedAvgComm`` / ``FedAvgRound`` - the framework's one comm-timing
    path (the device's comm stream, RCCL ordered after it, hipEvents on both streams) - so the bench's ``comm_ms``
    (each collective's own span) and ``comm_exposed_ms`` (the compute stream's stall on it) mean exactly what the
    FedAvg driver's CSV columns mean.  Per round, in enqueue order: launch the round's steps -> issue the
    all-reduce -> stage the NEXT round's batches (weight-independent) -> [next round] wait for the all-reduce ->
    launch.  ``none`` waits right after issuing (before the staging); ``tail`` waits only after the staging was
    enqueued, so the collective runs beside it.  ``collectives=False`` runs the same plan without any
    communication (the compute-only reference of the wall-clock exposure)."""

    def __init__(self, trainer, flat, ctx, overlap: str, allreduce=None, comm=None):
        from crossscale_ecg.parallel.overlap import FedAvgComm, FedAvgRound
        self.trainer, self.flat, self.ctx = trainer, flat, ctx
        self.overlap = overlap if ctx.distributed else "none"
        self.comm = comm or FedAvgComm(ctx, allreduce=allreduce)
        self.fround = FedAvgRound(flat, self.comm, self.overlap)
        self.syncs = 0
        self.collectives = True
        self.recs = []

    def run(self, plan, then=None):
        """``then``: size of the round that will follow ``plan`` (its batches are staged behind the last round)."""
        from crossscale_ecg.parallel.overlap import CommRecord
        for i, n in enumerate(plan):
            next_n = plan[i + 1] if i + 1 < len(plan) else then
            self.trainer.prepare_round(n, reset_loss=False)  # no-op when the previous round staged it
            self.fround.begin_round()  # tail: the next batches were staged while the all-reduce ran
            self.trainer.launch_round(n)
            if self.collectives:
                if self.ctx.distributed:
                    rec = CommRecord()
                    self.fround.end_round(rec)
                    self.recs.append(rec)
                self.syncs += 1
            if next_n is not None and hasattr(self.trainer, "stage"):
                self.trainer.stage(next_n)
        self.drain()

    def drain(self):
        self.fround.finalize()

    def comm_summary(self):
        """(comm_ms, exposed_ms) summed over the recorded rounds (call after a device synchronize)."""
        return (sum(r.comm_ms() for r in self.recs), sum(r.exposed_ms() for r in self.recs))


def weights_digest(flat):
    """float64 sum and abs-sum of the flat weights plus their first and last 8 values (18 numbers)."""
    f = flat.detach().double()
    return [float(f.sum()), float(f.abs().sum())] + f[:8].tolist() + f[-8:].tolist()


def torch_eager_rate(x, y, B, steps, device):
    import torch
    import torch.nn.functional as F
    from crossscale_ecg.models.tiny_ecg import TinyECG
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


def conv1d_speedup(device, B=256, L=500, K=7, trials=15, burst=20):
    """Module-2 comparison at one grid point.  ``once``: the reference's ``time_once`` (3 warm-up calls + ONE
    synchronised timed call, Module_2/benchmark_part_2.py:61-67), median over 15 trials; ``burst``: mean of
    ``burst`` back-to-back calls (secondary)."""
    import torch
    from crossscale_ecg.ops.conv1d import HipConv1dValid, conv1d_valid
    x = torch.randn(B, 1, L, device=device)
    w = torch.randn(K, device=device)
    conv = torch.nn.Conv1d(1, 1, K, bias=False).to(device)
    with torch.no_grad():
        conv.weight.copy_(w.view(1, 1, K))
    out = torch.empty(B, L - K + 1, device=device)

    def once(fn, sync=True):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if sync:  # the blocking HIP op returns with its output complete and needs none
            torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    def bursty(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(burst):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / burst

    x2 = x[:, 0].contiguous()
    op = HipConv1dValid(w, blocking=True)  # bound op: returns when its output is complete
    tfn = lambda: conv(x)  # noqa: E731
    hcall = lambda: op(x2, out)  # noqa: E731
    hfn = lambda: conv1d_valid(x2, w, backend="hip", out=out)  # noqa: E731  (async, for the burst timing)
    with torch.no_grad():
        ok = torch.allclose(hcall(), tfn()[:, 0], atol=1e-4, rtol=1e-4)
        t_once = [once(tfn) for _ in range(trials)]
        h_once = [once(hcall, sync=False) for _ in range(trials)]
        t_b = [bursty(tfn) for _ in range(trials)]
        h_b = [bursty(hfn) for _ in range(trials)]
    med = statistics.median
    return {"conv1d_torch_ms_median": round(med(t_once), 5), "conv1d_hip_ms_median": round(med(h_once), 5),
            "conv1d_speedup_vs_torch": round(med(t_once) / med(h_once), 3),
            "conv1d_burst_torch_ms": round(med(t_b), 5), "conv1d_burst_hip_ms": round(med(h_b), 5),
            "conv1d_burst_speedup_vs_torch": round(med(t_b) / med(h_b), 3), "conv1d_matches_torch": bool(ok)}


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse(argv)
    if a.gpus > 1 and not _under_launcher():
        return self_launch(a, argv)

    import torch
    sys.path.insert(0, ROOT)
    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.models.tiny_ecg import TinyECG, num_params
    from crossscale_ecg.parallel.env import (init_distributed, barrier, shutdown_distributed, rccl_init_log,
                                             rccl_transports, peer_access, rccl_log_env_restore, rccl_log_remove)

    # RCCL runs: its INIT log (channel -> transport) goes to a per-rank file read back after the run
    rccl_log = None
    if a.device == "gpu" and os.environ.get("ECG_DIST_BACKEND", "nccl") == "nccl" and \
            int(os.environ.get("WORLD_SIZE", "1")) > 1:
        rccl_log = rccl_init_log()
    ctx = init_distributed(prefer_gpu=a.device == "gpu")
    if rccl_log is not None:  # the communicator exists (eager device_id init): children must not inherit the log
        rccl_log_env_restore()
    if ctx.world_size != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={ctx.world_size}")
    dev = ctx.device
    on_gpu = dev.type == "cuda"
    placement = {"numa_node": -1, "cpus": "", "bound": False}
    if on_gpu and not a.no_numa_bind:  # this rank -> its slice of its GPU's NUMA-node CPUs (parallel/numa.py)
        from crossscale_ecg.parallel.numa import bind_to_gpu_numa
        placement = bind_to_gpu_numa(dev.index)
    if a.device == "gpu" and not on_gpu:
        raise SystemExit("bench.py needs a GPU (use --device cpu for the plumbing rehearsal)")
    if not on_gpu:
        a.backend, a.no_extras = "torch", True
    resnet = a.model.startswith("resnet")
    if a.batch_size is None:
        a.batch_size = 1024 if resnet else 256
    B, S = a.batch_size, a.local_steps

    def sync():
        if on_gpu:
            torch.cuda.synchronize(dev)

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
    if ctx.distributed:
        # round-0 broadcast of the global model (reference part3_fedavg_overlap_mpi_gpu.py:186) - also the first use
        # of the communicator - and one all-reduce of a scratch buffer of the weights' size, so RCCL's connection
        # set-up and first-collective costs stay out of the timed region even with --warmup 0
        from crossscale_ecg.parallel.fedavg import Communicator, broadcast_model, allreduce_mean_
        broadcast_model(Communicator(ctx), model)
        allreduce_mean_(torch.zeros_like(flat), ctx)
        sync()

    if resnet and a.backend == "fused":  # native ResNet step engine (one hipGraph per step)
        from crossscale_ecg.train.resnet_trainer import ResNetEngineTrainer
        trainer = ResNetEngineTrainer(model, x, y, B, S, lr=1e-2, momentum=0.9, seed=4321 + ctx.rank, ctx=ctx)
    elif a.backend == "fused":
        from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
        trainer = FusedTinyTrainer(model, x, y, B, S, lr=1e-2, momentum=0.9, seed=4321 + ctx.rank)
    else:
        from crossscale_ecg.train.local import TorchLocalTrainer
        amp = torch.bfloat16 if on_gpu else None
        trainer = TorchLocalTrainer(model, x, y, B, amp_dtype=amp, seed=4321 + ctx.rank)
    runner = FedAvgRunner(trainer, flat, ctx, a.overlap)
    # timing brackets: a shared-memory host barrier when every rank is on this node (parallel/host_barrier.py),
    # else the process-group barrier
    from crossscale_ecg.parallel.host_barrier import HostBarrier
    tbar = HostBarrier(ctx)

    timed_plan = round_plan(a.steps, S)
    warm_plan = round_plan(a.warmup, S) if a.warmup > 0 else []
    # One-time host work first - capture + upload of every round graph the warm-up and timed plans replay (the
    # warm-up replay inside prepare() is rolled back) and a full GC pass - THEN the warm-up rounds, so the timed
    # region starts right behind real training steps instead of after ~0.1 s of GPU idle (clocks and caches had
    # cooled: TinyECG K=20 13.1 -> 11.9 us/step wall, ResNet1D-34 3.44 -> 3.41 ms; profiles/r4/bench_order_ab.txt).
    if hasattr(trainer, "prepare"):
        trainer.prepare(sorted(set(timed_plan) | set(warm_plan)))
    gc.collect()
    if warm_plan:
        runner.run(warm_plan, then=timed_plan[0])
    runner.syncs = 0

    def bracket():  # synchronize + barrier (+ synchronize again only when the barrier itself enqueued GPU work)
        sync()
        tbar()
        if tbar.kind == "dist":
            sync()

    # device-side span of the timed work: hipEvents on the compute stream right after the opening bracket and
    # right after the last round was enqueued (the runner's drain made the compute stream wait for RCCL), so an
    # outlier can be attributed: gpu_ms ~ wall -> the GPU (or a starved queue) was slow; gpu_ms << wall -> host
    ev0 = ev1 = None
    if on_gpu:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(plan, then=None):
        """Wall seconds of ``plan`` between two brackets; no cyclic-GC pass inside (a collection there is host
        jitter, not work: one K=20 run measured 15.7 us/step wall at 11.4 us/step of GPU time; the full pass ran
        before the warm-up, the collector resumes right after the region)."""
        gc.disable()
        try:
            bracket()
            if ev0 is not None:  # recorded on the idle stream just before the clock starts (its host cost stays outside)
                ev0.record()
            t0 = time.perf_counter()
            runner.run(plan, then=then)
            if ev1 is not None:
                ev1.record()
            bracket()
            return time.perf_counter() - t0
        finally:
            gc.enable()

    # N>1: the same K steps once WITHOUT collectives first (untimed for the headline), so the wall-clock exposure of
    # the communication is measured on every backend as elapsed(with comm) - elapsed(compute only); the final
    # FedAvg of the timed region leaves every rank on identical weights again (checked below)
    solo_s = float("nan")
    if ctx.distributed:
        runner.collectives = False
        solo_s = timed(timed_plan, then=timed_plan[0])
        runner.collectives = True
    runner.recs.clear()
    runner.syncs = 0
    elapsed = timed(timed_plan)
    gpu_s = ev0.elapsed_time(ev1) / 1e3 if ev0 is not None else float("nan")
    comm_ms, exposed_ms = runner.comm_summary()
    exposed_wall_ms = max(0.0, (elapsed - solo_s) * 1e3) if solo_s == solo_s else 0.0
    digest = weights_digest(flat)  # after the last FedAvg all-reduce every rank must hold these exact weights
    tbar_kind = tbar.kind
    tbar.close()
    world_seen, dist_backend = 1, "none"
    per_rank = [[elapsed, gpu_s, comm_ms, exposed_ms, exposed_wall_ms]]
    placements = [placement]
    digests = [digest]
    links = None
    if ctx.distributed:
        import torch.distributed as dist
        world_seen, dist_backend = dist.get_world_size(), dist.get_backend()
        mine = torch.tensor([elapsed, gpu_s, comm_ms, exposed_ms, exposed_wall_ms], dtype=torch.float64,
                            device=dev if dist_backend == "nccl" else "cpu")
        allv = [torch.zeros_like(mine) for _ in range(world_seen)]
        dist.all_gather(allv, mine)
        per_rank = [[float(v) for v in t.tolist()] for t in allv]
        placements = [None] * world_seen
        dist.all_gather_object(placements, placement)
        dig = torch.tensor(digest, dtype=torch.float64, device=dev if dist_backend == "nccl" else "cpu")
        digs = [torch.zeros_like(dig) for _ in range(world_seen)]
        dist.all_gather(digs, dig)
        digests = [[float(v) for v in t.tolist()] for t in digs]
        links = [None] * world_seen
        dist.all_gather_object(links, {"transports": rccl_transports(rccl_log), "peer_access": peer_access(dev)})
        rccl_log_remove(rccl_log)
        elapsed = max(r[0] for r in per_rank)
        gpu_s = max(r[1] for r in per_rank)
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
            extras.update(conv1d_speedup(dev))
        except Exception as e:  # pragma: no cover
            extras["conv1d_error"] = repr(e)[:200]

    if ctx.rank == 0:
        n_par = sum(p.numel() for p in model.parameters())
        comm = "RCCL" if dist_backend == "nccl" else dist_backend
        rec = {
            "metric": METRIC if not resnet else "ECG samples/sec (node), ResNet1D-34 scaling-stress config (BASELINE config 5)",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": a.gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 5),
            "gpu_ms_per_step": round(gpu_s * 1e3 / a.steps, 5) if gpu_s == gpu_s else None,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic",
            "config": {
                "model": f"TinyECG ({num_params(2)} params)" if not resnet else f"{a.model} ({n_par} params)",
                "global_batch": B * a.gpus,
                "seq_len": a.win_len,
                "parallelism": f"dp{a.gpus}",
                "sync": f"fedavg every {S} local steps ({comm} all_reduce AVG, overlap={runner.overlap})",
                "per_client_batch": B,
                "max_windows_per_client": a.max_windows,
                "backend": a.backend,
            },
            "rccl_world_size": world_seen,
            "dist_backend": dist_backend,
            "fedavg_syncs_timed": runner.syncs,
            "timing_barrier": tbar_kind,
            "timed_round_plan": timed_plan if len(timed_plan) <= 4 else f"{len(timed_plan)} rounds",
            "final_avg_loss": round(loss, 6) if loss == loss else None,
            # per-rank diagnosis of the MAX: wall and GPU-event ms/step; the timed collectives' own span (comm_ms)
            # and the compute side's measured stall on them (comm_exposed_ms: compute-stream events on RCCL, host
            # time blocked in wait on host-staged gloo; parallel/overlap.py), summed over the timed rounds; and the
            # wall-clock exposure (comm_exposed_wall_ms = elapsed - elapsed of the same K steps without
            # collectives, any backend)
            "per_rank_ms_per_step": [round(r[0] * 1e3 / a.steps, 5) for r in per_rank],
            "per_rank_gpu_ms_per_step": [round(r[1] * 1e3 / a.steps, 5) if r[1] == r[1] else None for r in per_rank],
            "comm_ms": [round(r[2], 4) for r in per_rank],
            "comm_exposed_ms": [round(r[3], 4) for r in per_rank],
            "comm_exposed_wall_ms": [round(r[4], 4) for r in per_rank],
            "comm_timing": runner.comm.kind if ctx.distributed else "none",
            # rank -> NUMA node : CPU slice [split basis: kfd = planned over every GPU of the machine]
            "rank_cpus": [f"node{p.get('numa_node', -1)}:{p.get('cpus', '')}" + ("" if p.get("bound") else " (unbound)")
                          + (f" [{p['basis']}]" if p.get("basis") else "") for p in placements],
            # timing method: the cyclic GC is paused inside the timed region (restarted right after); the first
            # timed round's batch indices were drawn behind the last warmup round (later rounds' staging is timed)
            "gc_paused_in_timed_region": True,
            "first_round_staged_in_warmup": a.warmup > 0,
            # self-check of the FedAvg result: float64 sum / abs-sum and the first and last 8 weights of every rank
            # after the final all-reduce (must be bit-identical across ranks)
            "fedavg_weights_identical": all(d == digests[0] for d in digests),
            "fedavg_weights_checksum": digests[0][0],
            **({"rccl_links": links} if links is not None else {}),
            **extras,
        }
        print(json.dumps(rec), flush=True)
    if hasattr(trainer, "close"):
        trainer.close()
    barrier(ctx)
    shutdown_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
