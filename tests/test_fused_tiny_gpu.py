"""Numerics of the fused TinyECG HIP step vs a plain PyTorch fp32 reference of the same computation."""
import pytest
import torch
import torch.nn.functional as F

import crossscale_ecg  # noqa: F401
from crossscale_ecg.models.tiny_ecg import TinyECG, num_params

pytestmark = pytest.mark.gpu


def _setup(B=64, L=500, N=300, nc=2, seed=0, labels="random"):
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(N, L, generator=g).to(dev)
    if labels == "random":
        y = torch.randint(0, nc, (N,), generator=g).to(dev)
    else:
        y = torch.zeros(N, dtype=torch.long, device=dev)
    torch.manual_seed(seed)
    model = TinyECG(num_classes=nc).to(dev)
    idx = torch.randperm(N, generator=g)[:B].to(torch.int32).to(dev)
    return dev, x, y, model, idx


def _ref_grads(model, x, y, idx):
    m = TinyECG(num_classes=model.num_classes).to(x.device)
    m.load_state_dict(model.state_dict())
    sel = idx.long()
    loss = F.cross_entropy(m(x[sel].unsqueeze(1)), y[sel])
    loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    return g, loss.detach()


TOL = {"bf16": 2e-2, "fp32": 2e-5}


@pytest.mark.parametrize("precision,L", [("bf16", 500), ("bf16", 64), ("bf16", 333), ("bf16", 1000),
                                         ("fp32", 500), ("fp32", 64), ("fp32", 333)])
def test_forward_matches_torch(L, precision):
    from crossscale_ecg.ops.fused_tiny import tiny_forward
    dev, x, y, model, idx = _setup(L=L)
    flat = model.flatten_parameters()
    out = tiny_forward(flat, x, idx, idx.numel(), 2, precision=precision)
    ref = model(x[idx.long()].unsqueeze(1))
    torch.cuda.synchronize()
    err = (out - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-3
    assert err / scale < TOL[precision], f"max err {err} (scale {scale})"


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
@pytest.mark.parametrize("nc,L", [(2, 500), (5, 500), (2, 130)])
def test_step_grads_match_autograd(nc, L, precision):
    from crossscale_ecg.ops.fused_tiny import tiny_step_grads, reduce_slab, labels_int32
    dev, x, y, model, idx = _setup(nc=nc, L=L)
    gref, lref = _ref_grads(model, x, y, idx)
    flat = model.flatten_parameters()
    slab = tiny_step_grads(flat, x, labels_int32(y, nc), idx, idx.numel(), nc, precision=precision)
    grad, loss = reduce_slab(slab, nc)
    torch.cuda.synchronize()
    P = num_params(nc)
    assert grad.numel() == P
    assert abs(loss.item() / idx.numel() - lref.item()) < 1e-2 * max(1.0, abs(lref.item()))
    # per-tensor relative error (bf16 operands, fp32 accumulation)
    off = 0
    for name, p in model.named_parameters():
        n = p.numel()
        a, b = grad[off:off + n], gref[off:off + n]
        rel = (a - b).norm().item() / (b.norm().item() + 1e-6)
        assert rel < (3e-2 if precision == "bf16" else 1e-4), f"{name}: rel err {rel:.4g} |ref|={b.norm().item():.3e}"
        off += n


@pytest.mark.parametrize("precision", ["bf16", "fp32"])
def test_train_step_and_graph_match_torch_sgd(precision):
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    dev, x, y, model, idx = _setup(B=128, N=1024)
    ref = TinyECG().to(dev)
    ref.load_state_dict(model.state_dict())
    opt = torch.optim.SGD(ref.parameters(), lr=1e-2, momentum=0.9)
    tr = FusedTinyTrainer(model, x, y, batch_size=128, steps_per_round=4, seed=123, precision=precision)
    tr.run_round()  # graph path
    torch.cuda.synchronize()
    # replay the same batches through torch
    tab = tr.idx_table.clone()
    for s in range(4):
        sel = tab[s].long()
        opt.zero_grad()
        F.cross_entropy(ref(x[sel].unsqueeze(1)), y[sel]).backward()
        opt.step()
    got = tr.params[: num_params(2)]
    want = torch.cat([p.detach().reshape(-1) for p in ref.parameters()])
    rel = (got - want).norm().item() / want.norm().item()
    assert rel < (1e-3 if precision == "bf16" else 1e-5), rel
    # state_dict views the flat buffer
    sd = model.state_dict()
    assert torch.equal(sd["net.2.weight"].reshape(-1), tr.params[128:1408])
    tr.close()


def test_two_launch_round_is_deterministic():
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    outs = []
    for _ in range(2):
        dev, x, y, model, _ = _setup(B=256, N=2048)
        tr = FusedTinyTrainer(model, x, y, 256, 10, seed=11)
        tr.run_round()
        torch.cuda.synchronize()
        outs.append(tr.params.clone())
        tr.close()
    # atomics-free fixed-order reduction: bitwise reproducible run to run
    assert torch.equal(outs[0], outs[1])


def test_fp32_window_limit_is_reported():
    """fp32 activations take twice the LDS: windows beyond the fused limit fail loudly (op-by-op path)."""
    from crossscale_ecg.ops._lib import NativeError
    from crossscale_ecg.ops.fused_tiny import tiny_forward
    dev, x, y, model, idx = _setup(L=1000)
    with pytest.raises(NativeError):
        tiny_forward(model.flatten_parameters(), x, idx, idx.numel(), 2, precision="fp32")


def test_graph_equals_eager():
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    dev, x, y, model, _ = _setup(B=64, N=640)
    m2 = TinyECG().to(dev)
    m2.load_state_dict(model.state_dict())
    a = FusedTinyTrainer(model, x, y, 64, 5, seed=7, use_graph=True)
    b = FusedTinyTrainer(m2, x, y, 64, 5, seed=7, use_graph=False)
    for _ in range(3):
        a.run_round()
        b.run_round()
    torch.cuda.synchronize()
    assert torch.allclose(a.params, b.params, rtol=1e-5, atol=1e-6)
    assert abs(a.avg_loss() - b.avg_loss()) < 1e-4
    a.close()
    b.close()


def test_training_reduces_loss_on_learnable_labels():
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    x = torch.randn(4096, 500, device=dev) + torch.randn(4096, 1, device=dev) * 0.5
    y = (x.mean(1) > 0).long()
    model = TinyECG().to(dev)
    tr = FusedTinyTrainer(model, x, y, 256, 50, lr=5e-2, seed=0)
    tr.run_round()
    first = tr.avg_loss()
    for _ in range(6):
        tr.run_round()
    last = tr.avg_loss()
    assert last < first * 0.9, (first, last)
    tr.close()


def test_prepare_rollback_and_staged_rounds_bitwise():
    """``prepare`` (capture + upload + one warm replay) leaves no trace in the training state, and staging the next
    round's batches behind the current round (``next_n``) gives bit-identical training to staging at launch."""
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    plan = [5, 5, 3, 5, 2]
    outs = []
    for mode in ("plain", "prepared_staged"):
        dev, x, y, model, _ = _setup(B=64, N=1024)
        tr = FusedTinyTrainer(model, x, y, 64, 5, seed=21)
        if mode == "plain":
            for n in plan:
                tr.run_round(n, reset_loss=False)
        else:
            tr.prepare(sorted(set(plan)))
            for i, n in enumerate(plan):
                tr.run_round(n, reset_loss=False, next_n=plan[i + 1] if i + 1 < len(plan) else None)
        torch.cuda.synchronize()
        outs.append((tr.params.clone(), tr.mom.clone(), tr.avg_loss(), tr.idx_table.clone()))
        tr.close()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert outs[0][2] == outs[1][2] and torch.equal(outs[0][3][:2], outs[1][3][:2])


@pytest.mark.parametrize("B", [16, 256])
def test_prefrag_grads_bitwise_equal_lds_path(B):
    """Prepared-fragment kernel (conv operands from the global image) == LDS-built operands, bit for bit, for the
    gradient slab and the forward logits."""
    from crossscale_ecg.ops.fused_tiny import tiny_step_grads, tiny_forward, labels_int32
    dev, x, y, model, idx = _setup(B=B, N=max(4 * B, 64))
    flat = model.flatten_parameters()
    y32 = labels_int32(y, 2)
    from crossscale_ecg.models.tiny_ecg import num_params
    P = num_params(2)  # columns [0, P]: gradient row + loss (the slab's padding columns are never written)
    a = tiny_step_grads(flat, x, y32, idx, idx.numel(), 2, prefrag=True)[:, :P + 1]
    b = tiny_step_grads(flat, x, y32, idx, idx.numel(), 2, prefrag=False)[:, :P + 1]
    torch.cuda.synchronize()
    d = (a - b).abs()
    assert torch.equal(a, b), (d.max().item(), (d.amax(0) > 0).nonzero().flatten()[:20].tolist(),
                               (d.amax(1) > 0).nonzero().flatten().tolist())
    fa = tiny_forward(flat, x, idx, idx.numel(), 2, prefrag=True)
    fb = tiny_forward(flat, x, idx, idx.numel(), 2, prefrag=False)
    assert torch.equal(fa, fb)


@pytest.mark.parametrize("graph", [True, False])
def test_prefrag_round_graph_bitwise_equal_lds_eager_with_external_updates(graph):
    """PF round graphs (image rebuilt by the graph's first node, kept by every step's SGD epilogue) reproduce the
    LDS-built eager steps bit for bit over several rounds - also after the weights are rewritten between rounds
    (what a FedAvg all-reduce / broadcast does)."""
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    dev, x, y, model, _ = _setup(B=128, N=1024)
    m2 = TinyECG().to(dev)
    m2.load_state_dict(model.state_dict())
    a = FusedTinyTrainer(model, x, y, 128, 7, seed=9, use_graph=graph, prefrag=True)
    b = FusedTinyTrainer(m2, x, y, 128, 7, seed=9, use_graph=False, prefrag=False)
    assert a.prefrag and not b.prefrag
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    for r in range(4):
        a.run_round()
        b.run_round()
        if r == 1:  # external rewrite of the weights between rounds
            noise = torch.randn(a.params.shape, device=dev, generator=g) * 1e-2
            a.params.add_(noise)
            b.params.add_(noise)
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params), (a.params - b.params).abs().max()
    assert torch.equal(a.mom, b.mom)
    assert a.avg_loss() == b.avg_loss()
    a.close()
    b.close()


@pytest.mark.parametrize("L,B", [(500, 128), (250, 96)])  # 16-byte rows / scalar rows (L % 4 != 0)
def test_gather_round_graph_bitwise_equal_plain(L, B):
    """PF round graphs whose reduce launches gather the next step's windows and labels (``gather``) == the
    plain PF graph and the eager C++ step loop, bit for bit, over full and partial rounds (1-step rounds gather
    nothing; odd and even step counts end on either ping-pong buffer)."""
    from crossscale_ecg.ops.fused_tiny import FusedTinyTrainer
    plan = [7, 1, 2, 3, 7, 4]
    outs = []
    for gather, graph in ((True, True), (False, True), (False, False)):
        dev, x, y, model, _ = _setup(B=B, L=L, N=1024, nc=5)
        tr = FusedTinyTrainer(model, x, y, B, 7, seed=21, prefrag=True, use_graph=graph)
        tr.gather = gather
        if gather and tr.xg is None:
            tr.xg = torch.zeros(2 * B * ((L + 3) // 4 * 4), dtype=torch.float32, device=dev)
            tr.yg = torch.zeros(2 * B, dtype=torch.int32, device=dev)
        tr.prepare(sorted(set(plan)))
        for i, n in enumerate(plan):
            tr.run_round(n, reset_loss=False, next_n=plan[i + 1] if i + 1 < len(plan) else None)
        torch.cuda.synchronize()
        outs.append((tr.params.clone(), tr.mom.clone(), tr.avg_loss()))
        if gather:  # the last round (4 steps) ran its step 3 on buffer 1, gathered from that step's batch rows
            rows = tr.idx_table[3].long()
            ldg = (L + 3) // 4 * 4
            assert torch.equal(tr.yg[B:], tr.y32[rows])
            assert torch.equal(tr.xg.view(2, B, ldg)[1, :, :L], tr.x[rows])
        tr.close()
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0]) and torch.equal(outs[0][1], o[1])
        assert outs[0][2] == o[2]
