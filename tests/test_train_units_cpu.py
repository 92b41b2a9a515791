"""CPU unit tests of the eager training pieces the reference's G0 / G1 loops map to (train/steps.py, the
per-client trainer train/local.py) and of the timers (utils/timing.py)."""
import copy
import time

import torch
import torch.nn.functional as F

import crossscale_ecg  # noqa: F401
from crossscale_ecg.models.tiny_ecg import TinyECG
from crossscale_ecg.train.local import TorchLocalTrainer
from crossscale_ecg.train.steps import make_scaler, train_step_G0, train_step_G1
from crossscale_ecg.utils.timing import WallTimer, warm_until_stable


def _data(n=64, L=128, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 1, L, generator=g), torch.randint(0, 2, (n,), generator=g)


def test_g0_step_equals_manual_sgd_step():
    """train_step_G0 (reference part3_mpi_gpu_train.py G0: fp32 forward / CE / backward / SGD step) == the same
    update written out by hand."""
    torch.manual_seed(0)
    m = TinyECG()
    ref = copy.deepcopy(m)
    x, y = _data()
    opt = torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9)
    loss = train_step_G0(m, x, y, opt, "cpu")
    ref.zero_grad()
    l_ref = F.cross_entropy(ref(x), y)
    l_ref.backward()
    with torch.no_grad():
        for p in ref.parameters():
            p -= 0.05 * p.grad  # first momentum step: buffer = grad
    assert abs(loss - l_ref.item()) < 1e-6
    for a, b in zip(m.parameters(), ref.parameters()):
        assert torch.allclose(a, b, atol=1e-6)


def test_g1_step_bf16_autocast_trains_and_needs_no_scaler_on_cpu():
    """G1 (AMP) with bf16 autocast: no GradScaler (bf16 has fp32's exponent range); a few steps reduce the loss on a
    fixed batch."""
    torch.manual_seed(1)
    m = TinyECG()
    x, y = _data(seed=1)
    assert make_scaler("cpu", torch.bfloat16) is None
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    first = train_step_G1(m, x, y, opt, None, "cpu", amp_dtype=torch.bfloat16)
    for _ in range(30):
        last = train_step_G1(m, x, y, opt, None, "cpu", amp_dtype=torch.bfloat16)
    assert last < first
    assert isinstance(train_step_G1(m, x, y, opt, None, "cpu", sync=False), torch.Tensor)


def test_torch_local_trainer_round_api():
    """TorchLocalTrainer: the round API bench.py drives (prepare_round / launch_round / avg_loss) counts steps and
    averages the loss over the window; momentum reset zeroes the buffers."""
    torch.manual_seed(2)
    x = torch.randn(200, 128)
    y = torch.randint(0, 2, (200,))
    tr = TorchLocalTrainer(TinyECG(), x, y, 16, amp_dtype=None, seed=3)
    tr.prepare_round(5)
    tr.launch_round(5)
    assert tr.steps_done == 5 and tr._loss_steps == 5
    a = tr.avg_loss()
    assert 0.0 < a < 5.0
    tr.run_round(3)
    assert tr.steps_done == 8 and tr._loss_steps == 3
    tr.reset_momentum()
    assert all(float(st["momentum_buffer"].abs().sum()) == 0.0 for st in tr.opt.state.values())


def test_timers():
    t = WallTimer()
    with t():
        time.sleep(0.01)
    assert t.ms >= 9.0
    calls = []
    n = warm_until_stable(lambda: calls.append(1), min_steps=3, window=3, max_steps=50)
    assert 3 <= n <= 50 and len(calls) == n
