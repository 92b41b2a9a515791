"""RCCL (torch.distributed "nccl") multi-GPU suite: one process per GPU, one GPU per rank.

Skipped unless at least 2 GPUs are visible (the driver's 8-GPU node runs it at world 2 and at world
min(8, #GPUs)).  Mirrors tests/test_dist_gloo.py and tests/test_resnet_trainer_gpu.py on the real transport
(SURVEY §4.3): flat AVG all-reduce == mean, broadcast, delayed FedAvg, weighted/dropout averaging, exact tail
overlap == none (TinyECG fused client and ResNet engine), DDP segment all-reduce, the fused-TinyECG DDP round,
a 2-round ``run_fedavg`` with CSV rows for every rank, and ``bench.py --gpus N`` self-launch.
"""
import csv
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_GPU = torch.cuda.device_count() if torch.cuda.is_available() else 0
need2 = pytest.mark.skipif(N_GPU < 2, reason="needs >= 2 GPUs (one RCCL rank per GPU)")
WORLDS = sorted({2, min(8, N_GPU)}) if N_GPU >= 2 else [2]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.parallel import env as penv
    penv._CTX = None
    ctx = penv.init_distributed(backend="nccl")
    try:
        assert ctx.backend == "nccl" and ctx.device == torch.device("cuda", rank)
        res = globals()[case](ctx)
        torch.save(res, os.path.join(out_dir, f"{case}_{rank}.pt"))
    finally:
        penv.shutdown_distributed()


def _run(world, case, tmp_path):
    mp.start_processes(_worker, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    return [torch.load(tmp_path / f"{case}_{r}.pt", weights_only=True) for r in range(world)]


# ----------------------------------------------------------------------------------------------- cases
def case_avg_and_bcast(ctx):
    import torch.distributed as dist
    from crossscale_ecg.models.tiny_ecg import TinyECG
    from crossscale_ecg.parallel.fedavg import Communicator, fedavg_allreduce, broadcast_model
    torch.manual_seed(100 + ctx.rank)
    m = TinyECG().to(ctx.device)
    m.flatten_parameters()
    before = m.flat.clone()
    allb = [torch.zeros_like(before) for _ in range(ctx.world_size)]
    dist.all_gather(allb, before)
    comm = Communicator(ctx)
    fedavg_allreduce(comm, m)
    ok_mean = torch.allclose(m.flat, torch.stack(allb).mean(0), atol=1e-6)
    with torch.no_grad():
        m.flat.add_(ctx.rank)
    broadcast_model(comm, m)
    g = [torch.zeros_like(m.flat) for _ in range(ctx.world_size)]
    dist.all_gather(g, m.flat)
    ok_bcast = all(torch.equal(g[0], t) for t in g)
    v = comm.allreduce(float(ctx.rank), "sum")
    rows = comm.gather({"rank": ctx.rank}, root=0)
    ok_comm = v == sum(range(ctx.world_size)) and (ctx.rank != 0 or [r["rank"] for r in rows] == list(range(ctx.world_size)))
    return torch.tensor([ok_mean, ok_bcast, ok_comm])


def case_delayed_and_weighted(ctx):
    from crossscale_ecg.parallel.fedavg import DelayedFedAvg, weighted_fedavg_
    flat = torch.full((4,), float(ctx.rank), device=ctx.device)
    d = DelayedFedAvg(flat, ctx)
    d.boundary()
    flat.add_(10.0)
    d.boundary()
    mean = (ctx.world_size - 1) / 2.0
    ok1 = torch.allclose(flat, torch.full((4,), mean + 10.0, device=ctx.device))
    d.finalize()
    f2 = torch.full((8,), float(ctx.rank + 1), device=ctx.device)
    w = 0.0 if ctx.rank == 0 else float(ctx.rank)
    total = weighted_fedavg_(f2, w, ctx)
    ws = [0.0] + [float(r) for r in range(1, ctx.world_size)]
    expect = sum(wi * (r + 1) for r, wi in enumerate(ws)) / sum(ws)
    ok2 = abs(total - sum(ws)) < 1e-6 and torch.allclose(f2, torch.full((8,), expect, device=ctx.device))
    return torch.tensor([ok1, ok2])


def _tiny_client(ctx, steps):
    from crossscale_ecg.models.tiny_ecg import TinyECG
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    g = torch.Generator(device=ctx.device)
    g.manual_seed(1337 + ctx.rank)
    x = torch.randn(2048, 500, generator=g, device=ctx.device)
    y = (x.mean(1) > 0).long()
    torch.manual_seed(0)
    m = TinyECG().to(ctx.device)
    return m, FusedTinyTrainer(m, x, y, 64, steps, seed=7 + ctx.rank)


SPIN = 2_000_000  # GPU cycles (~1 ms) of weight-independent work in each round's preparation
SPIN_MS_MIN = 0.5  # a lower bound of that preparation's duration


def _tiny_fedavg(ctx, mode, spin=0):
    from crossscale_ecg.parallel.overlap import CommRecord, FedAvgComm, FedAvgRound
    m, tr = _tiny_client(ctx, 5)
    comm = FedAvgComm(ctx)
    fr = FedAvgRound(m.flat, comm, mode)
    recs = []

    def prep():
        tr.prepare_round(5)
        if spin:
            torch.cuda._sleep(spin)  # compute-stream work that reads no weights

    for _ in range(3):
        fr.begin_round(prep=prep)
        tr.launch_round(5)
        rec = CommRecord()
        fr.end_round(rec)
        recs.append(rec)
    fr.finalize()
    torch.cuda.synchronize()
    times = torch.tensor([[r.comm_ms(), r.exposed_ms()] for r in recs])
    out = m.flat.detach().cpu().clone()
    tr.close()
    return out, times


def case_tiny_tail_vs_none(ctx):
    a, ta = _tiny_fedavg(ctx, "none")
    b, tb = _tiny_fedavg(ctx, "tail")
    return torch.cat([a, b]), torch.cat([ta, tb])


def case_tiny_exposure(ctx):
    """[comm_ms, exposed_ms] per round for none / tail / delayed with a ~1 ms weight-independent preparation."""
    return [_tiny_fedavg(ctx, mode, SPIN)[1] for mode in ("none", "tail", "delayed")]


def case_resnet_tail_exposure(ctx):
    """The ResNet per-bucket tail: [comm_ms, exposed_ms] of the tail step's collectives."""
    from crossscale_ecg.models.resnet1d import resnet1d18
    from crossscale_ecg.parallel.overlap import CommRecord, FedAvgComm
    from crossscale_ecg.train.resnet_trainer import ResNetEngineTrainer
    torch.manual_seed(0)
    m = resnet1d18().to(ctx.device)
    x = torch.randn(512, 500, device=ctx.device)
    y = (x.mean(1) > 0).long()
    tr = ResNetEngineTrainer(m, x, y, 128, 3, seed=ctx.rank, ctx=ctx, bucket_mb=1.0)
    tr.run_round(2)
    comm, rec = FedAvgComm(ctx), CommRecord()
    tr.tail_fedavg(comm, rec)
    torch.cuda.synchronize()
    out = torch.tensor([rec.comm_ms(), rec.exposed_ms(), float(len(tr.issue_log))])
    tr.close()
    return out


def case_tiny_ddp_round(ctx):
    from crossscale_ecg.train.fedavg import _ddp_fused_round
    m, tr = _tiny_client(ctx, 4)
    tr.prepare_round(4)
    _ddp_fused_round(tr, ctx, 4)
    torch.cuda.synchronize()
    out = m.flat.detach().cpu().clone()
    tr.close()
    return out


def _resnet(ctx, mode):
    from crossscale_ecg.models.resnet1d import resnet1d18
    from crossscale_ecg.parallel.fedavg import fedavg_allreduce, Communicator
    from crossscale_ecg.train.resnet_trainer import ResNetEngineTrainer
    torch.manual_seed(0)
    m = resnet1d18().to(ctx.device)
    g = torch.Generator(device=ctx.device)
    g.manual_seed(100 + ctx.rank)
    x = torch.randn(128, 500, generator=g, device=ctx.device)
    y = (x.mean(1) > 0).long()
    tr = ResNetEngineTrainer(m, x, y, 16, 3, lr=0.05, seed=ctx.rank, ctx=ctx, sync="ddp" if mode == "ddp" else "fedavg")
    if mode == "ddp":
        tr.run_round(3)
    elif mode == "tail":
        tr.run_round(2)
        tr.tail_fedavg()
    else:
        tr.run_round(3)
        fedavg_allreduce(Communicator(ctx), m)
    torch.cuda.synchronize()
    keep = m._space.param_numel if mode == "ddp" else m.flat.numel()
    out = m.flat[:keep].detach().cpu().clone()
    tr.close()
    return out


def case_resnet_modes(ctx):
    return [_resnet(ctx, mode) for mode in ("ddp", "tail", "none")]


# ----------------------------------------------------------------------------------------------- tests
@need2
@pytest.mark.parametrize("world", WORLDS)
def test_rccl_avg_broadcast_gather(world, tmp_path):
    for res in _run(world, "case_avg_and_bcast", tmp_path):
        assert bool(res.all()), res


@need2
def test_rccl_delayed_and_weighted(tmp_path):
    for res in _run(2, "case_delayed_and_weighted", tmp_path):
        assert bool(res.all()), res


@need2
@pytest.mark.parametrize("world", WORLDS)
def test_rccl_tiny_tail_equals_none(world, tmp_path):
    outs = _run(world, "case_tiny_tail_vs_none", tmp_path)
    P = outs[0][0].numel() // 2
    for w, t in outs:
        assert torch.equal(w[:P], w[P:])  # tail == none, bit for bit
        assert torch.equal(w[:P], outs[0][0][:P])  # every client holds the averaged model
        assert bool((t >= 0).all())


@need2
def test_rccl_overlap_exposure(tmp_path):
    """``comm_ms`` is each collective's own span on the comm stream (issue after the weights are final -> RCCL done)
    and ``exposed_ms`` the compute stream's measured stall on it (parallel/overlap.py).  none: the compute stream
    waits right away, so it stalls for the whole collective; tail: the collective runs under the next round's ~1 ms
    preparation, so the stall is ~0 - at most what the preparation did not cover (rank skew can stretch a
    collective past it); delayed: it runs under a whole local round, the same bound."""
    def hidden(comm, exposed):
        return exposed <= 0.05 + 0.1 * comm + max(0.0, comm - SPIN_MS_MIN)

    for none, tail, delayed in _run(2, "case_tiny_exposure", tmp_path):
        for comm, exposed in none.tolist():
            assert comm > 0 and exposed >= 0.8 * comm - 0.05, (comm, exposed)
        for comm, exposed in tail[:-1].tolist():  # the last round's collective is drained by finalize()
            assert comm > 0 and hidden(comm, exposed), (comm, exposed)
        for comm, exposed in delayed[1:].tolist():
            assert comm > 0 and hidden(comm, exposed), (comm, exposed)


@need2
def test_rccl_resnet_bucket_tail_exposure(tmp_path):
    for comm, exposed, buckets in (t.tolist() for t in _run(2, "case_resnet_tail_exposure", tmp_path)):
        assert buckets > 4 and comm > 0 and exposed < comm, (comm, exposed, buckets)


@need2
def test_rccl_tiny_ddp_round(tmp_path):
    outs = _run(2, "case_tiny_ddp_round", tmp_path)
    assert torch.equal(outs[0], outs[1])


@need2
def test_rccl_resnet_ddp_tail_none(tmp_path):
    outs = _run(2, "case_resnet_modes", tmp_path)
    for i in range(3):
        assert torch.equal(outs[0][i], outs[1][i])
    assert torch.allclose(outs[0][1], outs[0][2], rtol=1e-5, atol=1e-6)  # tail == none up to summation order


def _torchrun(world, script, *args, timeout=600):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, script), *args]
    r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:]
    return r.stdout


@need2
@pytest.mark.parametrize("world", WORLDS)
def test_rccl_run_fedavg_csv(world, tmp_path):
    csv_path = tmp_path / "fedavg.csv"
    _torchrun(world, "part3_fedavg_overlap_mpi_gpu.py", "--synthetic-windows", "4096", "--rounds", "2",
              "--local-steps", "5", "--config", "both", "--overlap", "tail", "--results-csv", str(csv_path), "--quiet")
    rows = list(csv.DictReader(open(csv_path)))
    assert len(rows) == 2 * world * 2
    assert {int(r["world_size"]) for r in rows} == {world}
    assert {int(r["rank"]) for r in rows} == set(range(world))
    assert {r["backend"] for r in rows} == {"fused"}


@need2
def test_bench_self_launch_two_gpus():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "60", "--warmup",
                        "20", "--no-extras"], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["rccl_world_size"] == 2 and rec["dist_backend"] == "nccl"
    assert rec["fedavg_syncs_timed"] == 2 and rec["config"]["global_batch"] == 512
