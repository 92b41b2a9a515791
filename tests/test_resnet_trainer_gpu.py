"""ResNet1D FedAvg client on the native engine: run_fedavg integration (world 1), and 2 ranks sharing one GPU
over gloo for the DDP (segment all-reduce) and ``--overlap tail`` paths."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

import crossscale_ecg  # noqa: F401

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    from crossscale_ecg.config import FedAvgConfig
    base = dict(model="resnet1d18", config="G1", amp_dtype="bf16", batch_size=32, local_steps=3, rounds=2,
                synthetic_windows=256, max_windows=256, labels="parity", quiet=True, results_csv="", jsonl="")
    base.update(kw)
    return FedAvgConfig(**base)


def test_run_fedavg_resnet_engine_world1():
    from crossscale_ecg.parallel.env import init_distributed, shutdown_distributed
    from crossscale_ecg.train.fedavg import run_fedavg
    ctx = init_distributed(backend="gloo", prefer_gpu=True)
    try:
        rows = run_fedavg(_cfg(), ctx)
    finally:
        shutdown_distributed()
    assert len(rows) == 2 and all(r["backend"] == "hip" for r in rows)
    assert all(torch.isfinite(torch.tensor(r["avg_loss"])) for r in rows)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, out_dir, bucket_mb=4.0, tag=""):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.models.resnet1d import resnet1d18
    from crossscale_ecg.parallel.env import init_distributed, shutdown_distributed
    from crossscale_ecg.parallel.fedavg import fedavg_allreduce, Communicator
    from crossscale_ecg.train.resnet_trainer import ResNetEngineTrainer
    ctx = init_distributed(backend="gloo", prefer_gpu=True)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    m = resnet1d18().to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(100 + rank)
    x = torch.randn(128, 500, generator=g, device=dev)
    y = (x.mean(1) > 0).long()
    tr = ResNetEngineTrainer(m, x, y, 16, 3, lr=0.05, seed=rank, ctx=ctx, sync="ddp" if mode == "ddp" else "fedavg",
                             bucket_mb=bucket_mb)
    if mode == "ddp":
        tr.run_round(3)
    elif mode == "tail":
        tr.run_round(2)
        tr.tail_fedavg()
    else:  # none: 3 steps then one flat all-reduce
        tr.run_round(3)
        fedavg_allreduce(Communicator(ctx), m)
    torch.cuda.synchronize()
    # DDP keeps BN running statistics per client (like torch DDP without SyncBN): compare parameters only
    keep = m._space.param_numel if mode == "ddp" else m.flat.numel()
    torch.save(m.flat[:keep].detach().cpu(), os.path.join(out_dir, f"{mode}{tag}_{rank}.pt"))
    if rank == 0 and tr.issue_log:
        torch.save(torch.tensor([list(t) for t in tr.issue_log]), os.path.join(out_dir, f"{mode}{tag}_log.pt"))
    tr.close()
    shutdown_distributed()


@pytest.mark.parametrize("mode", ["ddp", "tail", "none"])
def test_two_clients_one_gpu(mode, tmp_path):
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, mode, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    a = torch.load(tmp_path / f"{mode}_0.pt", weights_only=True)
    b = torch.load(tmp_path / f"{mode}_1.pt", weights_only=True)
    assert torch.equal(a, b)  # every client holds the same (averaged) model


def test_tail_equals_none(tmp_path):
    for mode in ("tail", "none"):
        port = _free_port()
        mp.start_processes(_worker, args=(2, port, mode, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    a = torch.load(tmp_path / "tail_0.pt", weights_only=True)
    b = torch.load(tmp_path / "none_0.pt", weights_only=True)
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)


def test_ddp_buckets_equal_single_allreduce(tmp_path):
    """Bucketed DDP (~1 MB buckets: many collectives, issued while the backward runs) gives bitwise the weights of
    one all-reduce of the whole gradient (a bucket larger than the model)."""
    for tag, mb in (("_b1", 1.0), ("_all", 1e6)):
        port = _free_port()
        mp.start_processes(_worker, args=(2, port, "ddp", str(tmp_path), mb, tag), nprocs=2, join=True,
                           start_method="spawn")
    a = torch.load(tmp_path / "ddp_b1_0.pt", weights_only=True)
    b = torch.load(tmp_path / "ddp_all_0.pt", weights_only=True)
    assert torch.equal(a, b)
    log_b = torch.load(tmp_path / "ddp_b1_log.pt", weights_only=True)
    log_all = torch.load(tmp_path / "ddp_all_log.pt", weights_only=True)
    assert log_all.shape[0] == 3 and log_b.shape[0] > log_all.shape[0]  # 3 steps x 1 bucket vs many
