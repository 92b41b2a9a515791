"""Sequence-parallel TinyECG (time-sharded record, halo exchange over gloo) vs the single-process model."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import crossscale_ecg  # noqa: F401
from crossscale_ecg.parallel.seqpar import shard_bounds

from test_dist_gloo import _free_port

L_REC = 1531  # not a multiple of the world size: uneven shards


def _reference():
    from crossscale_ecg.models.tiny_ecg import TinyECG
    torch.manual_seed(7)
    m = TinyECG()
    x = torch.randn(3, 1, L_REC)
    y = torch.tensor([0, 1, 1])
    return m, x, y


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from crossscale_ecg.parallel.seqpar import SeqParallelTinyECG, allreduce_seq_grads_
        m, x, y = _reference()
        s, e = shard_bounds(L_REC, world, rank)
        sp = SeqParallelTinyECG(m)
        logits = sp(x[..., s:e], L_REC)
        loss = torch.nn.functional.cross_entropy(logits, y)
        loss.backward()
        allreduce_seq_grads_(m)
        # numpy copies travel by value (a tensor would travel as a shared-memory handle that dies with this process)
        q.put((rank, "ok", (logits.detach().numpy().copy(),
                            {n: p.grad.detach().numpy().copy() for n, p in m.named_parameters()})))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_shard_bounds_cover_record():
    for L, w in ((10, 3), (1531, 4), (7, 7)):
        spans = [shard_bounds(L, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == L
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1


def test_single_rank_matches_model():
    from crossscale_ecg.parallel.seqpar import SeqParallelTinyECG
    m, x, _ = _reference()
    assert torch.allclose(SeqParallelTinyECG(m)(x, L_REC), m(x), atol=1e-6)


@pytest.mark.parametrize("world", [2, 3])
def test_seq_parallel_matches_full_record(world):
    m, x, y = _reference()
    ref_logits = m(x)
    torch.nn.functional.cross_entropy(ref_logits, y).backward()
    ref_grads = {n: p.grad.clone() for n, p in m.named_parameters()}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        rank, status, res = q.get(timeout=240)
        assert status == "ok", res
        out[rank] = res
    for p in ps:
        p.join(timeout=60)
    for rank, (logits, grads) in out.items():
        logits = torch.from_numpy(logits)
        grads = {n: torch.from_numpy(g) for n, g in grads.items()}
        assert torch.allclose(logits, ref_logits.detach(), atol=1e-5), rank
        for n, g in grads.items():
            assert torch.allclose(g, ref_grads[n], atol=1e-5, rtol=1e-4), (rank, n, (g - ref_grads[n]).abs().max())
