"""Stream -> hardware-queue layout of an N > 1 rank, as a regression test on ONE GPU (profiles/r6/stream_queues.txt).

A world-1 RCCL group created exactly as ``parallel.env.init_distributed`` creates one (``nccl_pg_options``: RCCL's
internal stream from the high-priority pool) and the device's comm stream (``parallel.overlap.comm_stream``): an
all-reduce issued from the comm stream while a ~1.7 ms kernel runs on the compute stream must COMPLETE inside that
kernel's span.  With RCCL's stream on the compute stream's hardware queue (torch's default pool, measured in round 6)
the collective ran only after the compute kernel and this test fails.  Runs in a spawned process so the pytest
process keeps no process group.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    try:
        import torch.distributed as dist
        import crossscale_ecg  # noqa: F401
        from crossscale_ecg.parallel.env import nccl_pg_options
        from crossscale_ecg.parallel.overlap import comm_stream
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        opts = nccl_pg_options()
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev,
                                **({"pg_options": opts} if opts is not None else {}))
        comm = comm_stream(dev)
        compute = torch.cuda.current_stream(dev)
        buf = torch.ones(1458, device=dev)
        dist.all_reduce(buf, op=dist.ReduceOp.AVG)  # communicator warm-up
        torch.cuda.synchronize()
        res = []
        for _ in range(4):
            e0, e1, c1 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(compute)
            torch.cuda._sleep(4_000_000)  # ~1.7 ms on the compute stream
            e1.record(compute)
            with torch.cuda.stream(comm):
                buf.add_(1.0)
                dist.all_reduce(buf, op=dist.ReduceOp.AVG, async_op=True).wait()
                c1.record(comm)
            torch.cuda.synchronize()
            res.append((e0.elapsed_time(e1), e0.elapsed_time(c1)))
        dist.destroy_process_group()
        q.put(("ok", res, opts is not None))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put(("err", traceback.format_exc(), None))


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_rccl_collective_runs_beside_compute_kernel():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    status, res, high = q.get(timeout=240)
    p.join(timeout=60)
    assert status == "ok", res
    assert high, "ECG_RCCL_HIGH_PRIORITY must default to the high-priority RCCL stream"
    for compute_ms, comm_done_ms in res[1:]:  # the first iteration carries one-time costs
        assert comm_done_ms < 0.5 * compute_ms, (compute_ms, comm_done_ms, res)
