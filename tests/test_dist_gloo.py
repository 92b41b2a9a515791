"""Multi-process FedAvg / collectives on CPU with gloo (world 2 and 4), launcher env shim, entry points."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import crossscale_ecg  # noqa: F401
from crossscale_ecg.parallel import env as penv


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn_name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    penv._CTX = None
    torch.set_num_threads(1)
    try:
        ctx = penv.init_distributed(backend="gloo", prefer_gpu=False)
        res = globals()[fn_name](ctx)
        q.put((rank, "ok", res))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "err", traceback.format_exc()))
    finally:
        penv.shutdown_distributed()


def _run(world, fn_name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, fn_name, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        rank, status, res = q.get(timeout=240)
        assert status == "ok", res
        out[rank] = res
    for p in ps:
        p.join(timeout=60)
    return out


def case_fedavg_mean(ctx):
    from crossscale_ecg.models.tiny_ecg import TinyECG
    from crossscale_ecg.parallel.fedavg import Communicator, fedavg_allreduce, broadcast_model
    torch.manual_seed(100 + ctx.rank)
    m = TinyECG()
    m.flatten_parameters()
    before = m.flat.clone()
    comm = Communicator(ctx)
    allb = [torch.zeros_like(before) for _ in range(ctx.world_size)]
    dist.all_gather(allb, before)
    fedavg_allreduce(comm, m)
    expect = torch.stack(allb).mean(0)
    ok_mean = torch.allclose(m.flat, expect, atol=1e-6)
    # broadcast from rank 0 of a perturbed model
    with torch.no_grad():
        m.flat.add_(ctx.rank)
    broadcast_model(comm, m)
    g = [torch.zeros_like(m.flat) for _ in range(ctx.world_size)]
    dist.all_gather(g, m.flat)
    ok_bcast = all(torch.equal(g[0], t) for t in g)
    sd_ok = torch.equal(m.state_dict()["head.bias"], m.flat[1456:1458])
    return ok_mean and ok_bcast and sd_ok


def case_unflattened_model(ctx):
    from crossscale_ecg.parallel.fedavg import Communicator, fedavg_allreduce
    torch.manual_seed(ctx.rank)
    m = torch.nn.Linear(3, 2)
    w0 = m.weight.detach().clone()
    g = [torch.zeros_like(w0) for _ in range(ctx.world_size)]
    dist.all_gather(g, w0)
    fedavg_allreduce(Communicator(ctx), m)
    return torch.allclose(m.weight, torch.stack(g).mean(0), atol=1e-6)


def case_weighted_and_dropout(ctx):
    from crossscale_ecg.parallel.fedavg import weighted_fedavg_
    flat = torch.full((8,), float(ctx.rank + 1))
    w = 0.0 if ctx.rank == 0 else float(ctx.rank)
    total = weighted_fedavg_(flat, w, ctx)
    ws = [0.0] + [float(r) for r in range(1, ctx.world_size)]
    expect = sum(wi * (r + 1) for r, wi in enumerate(ws)) / sum(ws)
    return abs(total - sum(ws)) < 1e-6 and torch.allclose(flat, torch.full((8,), expect))


def case_delayed_fedavg(ctx):
    from crossscale_ecg.parallel.fedavg import DelayedFedAvg
    flat = torch.full((4,), float(ctx.rank))
    d = DelayedFedAvg(flat, ctx)
    d.boundary()            # round 0 ends: start avg of w_0 = rank
    flat.add_(10.0)         # round 1 local progress
    d.boundary()            # wait: w <- w + (avg_0 - w_0) = rank + 10 + (mean - rank)
    mean = (ctx.world_size - 1) / 2.0
    ok1 = torch.allclose(flat, torch.full((4,), mean + 10.0))
    d.finalize()
    return ok1


def case_communicator(ctx):
    from crossscale_ecg.parallel.fedavg import Communicator, mpi_avg
    c = Communicator(ctx)
    rows = c.gather({"rank": ctx.rank}, root=0)
    v = mpi_avg(c, float(ctx.rank))
    c.Barrier()
    ok = abs(v - (ctx.world_size - 1) / 2) < 1e-9
    if ctx.rank == 0:
        ok &= [r["rank"] for r in rows] == list(range(ctx.world_size))
    return ok


@pytest.mark.parametrize("world", [2, 4])
def test_fedavg_allreduce_and_broadcast(world):
    assert all(_run(world, "case_fedavg_mean").values())


def test_unflattened_model_path():
    assert all(_run(2, "case_unflattened_model").values())


def test_weighted_fedavg_with_dropped_client():
    assert all(_run(3, "case_weighted_and_dropout").values())


def test_delayed_overlap_semantics():
    assert all(_run(2, "case_delayed_fedavg").values())


def test_communicator_gather_and_avg():
    assert all(_run(2, "case_communicator").values())


def test_launcher_env_shim():
    env = {"OMPI_COMM_WORLD_RANK": "3", "OMPI_COMM_WORLD_SIZE": "8", "OMPI_COMM_WORLD_LOCAL_RANK": "3"}
    assert penv.apply_launcher_env_shim(env) == "OMPI"
    assert (env["RANK"], env["WORLD_SIZE"], env["LOCAL_RANK"]) == ("3", "8", "3")
    env = {"SLURM_PROCID": "1", "SLURM_NTASKS": "2", "SLURM_LOCALID": "0"}
    assert penv.apply_launcher_env_shim(env) == "SLURM"
    assert env["RANK"] == "1" and env["MASTER_ADDR"] == "127.0.0.1"
    env = {"RANK": "0", "WORLD_SIZE": "1", "PMI_RANK": "5"}
    assert penv.apply_launcher_env_shim(env) is None and env["RANK"] == "0"


def case_host_barrier(ctx):
    import time
    from crossscale_ecg.parallel.host_barrier import HostBarrier
    os.environ["LOCAL_WORLD_SIZE"] = str(ctx.world_size)
    b = HostBarrier(ctx, timeout_s=60)
    kind = b.kind
    for _ in range(300):  # back-to-back generations must not run into each other
        b()
    # ordering: rank r arrives r * 0.15 s late; nobody may leave before the last arrival
    b()
    time.sleep(0.15 * ctx.rank)
    arrive = time.time()
    b()
    leave = time.time()
    t = torch.tensor([arrive, leave], dtype=torch.float64)
    ts = [torch.zeros(2, dtype=torch.float64) for _ in range(ctx.world_size)]
    dist.all_gather(ts, t)
    t0 = time.perf_counter()
    for _ in range(1000):
        b()
    per_call_us = (time.perf_counter() - t0) * 1e3
    b.close()
    return kind, max(x[0].item() for x in ts), min(x[1].item() for x in ts), per_call_us


@pytest.mark.parametrize("world", [2, 3])
def test_host_barrier_shm(world):
    """Shared-memory timing barrier (bench.py): all ranks agree on the shm path, no rank leaves before the last
    one arrived, and 1000 generations in a row stay in step."""
    out = _run(world, "case_host_barrier")
    for kind, last_arrival, first_leave, per_call_us in out.values():
        assert kind == "shm"
        assert first_leave >= last_arrival
        assert per_call_us < 5000  # 1000 calls: < 5 ms each even on an oversubscribed CI box


def case_host_barrier_timeout(ctx):
    import time
    from crossscale_ecg.parallel.host_barrier import HostBarrier
    os.environ["LOCAL_WORLD_SIZE"] = str(ctx.world_size)
    b = HostBarrier(ctx, timeout_s=1.0)
    assert b.kind == "shm"
    b()  # both meet once
    err = None
    if ctx.rank == 0:  # rank 1 never arrives at the second generation: rank 0 must give up, not hang
        t0 = time.time()
        try:
            b()
        except RuntimeError as e:
            err = (str(e)[:40], time.time() - t0)
    dist.barrier()  # (gloo) both ranks done before the segment is closed
    b.close()
    return err


def test_host_barrier_timeout():
    out = _run(2, "case_host_barrier_timeout")
    msg, waited = out[0]
    assert "host barrier failed" in msg and 0.9 < waited < 30
    assert out[1] is None


def test_rccl_init_log_env_restored_and_removed(tmp_path, monkeypatch):
    """advisor r5: the NCCL_DEBUG* variables set for the transport record do not leak to child processes, and the
    per-process INIT log is deleted once read."""
    from crossscale_ecg.parallel import env as penv
    for k in ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("NCCL_DEBUG_SUBSYS", "COLL")
    path = penv.rccl_init_log(str(tmp_path))
    assert os.environ["NCCL_DEBUG"] == "INFO" and os.environ["NCCL_DEBUG_FILE"] == path
    with open(path, "w") as f:
        f.write("x NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC\n")
    penv.rccl_log_env_restore()
    assert "NCCL_DEBUG" not in os.environ and "NCCL_DEBUG_FILE" not in os.environ
    assert os.environ["NCCL_DEBUG_SUBSYS"] == "COLL"
    assert penv.rccl_transports(path) == {"P2P/IPC": 1}
    penv.rccl_log_remove(path)
    assert not os.path.exists(path)


def case_comm_span_is_completion_time(ctx):
    """FedAvgComm host timing: comm_ms ends when the collective COMPLETED (its future's callback), not when the
    consumer looked; the host stall is only the time blocked in ``wait``."""
    import time
    from crossscale_ecg.parallel.overlap import CommRecord, FedAvgComm
    comm = FedAvgComm(ctx)
    t = torch.full((1458,), float(ctx.rank))
    out = []
    for _ in range(3):
        dist.barrier()
        rec = CommRecord()
        p = comm.issue(t, rec)
        time.sleep(0.05)  # 50 ms of weight-independent work before the consumer waits
        comm.wait([p], rec)
        out.append((rec.comm_ms(), rec.exposed_ms()))
    return comm.kind, out, float(t[0])


def test_fedavgcomm_host_span_and_stall():
    res = _run(2, "case_comm_span_is_completion_time")
    for kind, spans, v in res.values():
        assert kind == "host" and v == 0.5  # the average of ranks 0 and 1 (SUM + divide chained on the future)
        # the collective itself is far shorter than the 50 ms before the wait; nothing left to wait for
        assert sum(c for c, _ in spans) / len(spans) < 25.0, spans
        assert all(e < 5.0 for _, e in spans), spans
