"""MFMA multi-channel conv1d (channels-last) vs plain PyTorch fp32 F.conv1d: forward, dgrad, wgrad, bias."""
import os

import pytest
import torch
import torch.nn.functional as F

import crossscale_ecg  # noqa: F401

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

CASES = [  # B, L, Cin, Cout, K, stride, pad
    (4, 125, 64, 64, 3, 1, 1),
    (3, 125, 64, 128, 3, 2, 1),
    (2, 63, 128, 128, 3, 1, 1),
    (5, 33, 128, 256, 1, 2, 0),
    (2, 16, 512, 512, 3, 1, 1),
    (3, 70, 64, 192, 5, 1, 2),
    (2, 32, 256, 512, 3, 2, 1),  # (L+2p-K) % stride != 0: last input row only reached by one tap
    (3, 32, 256, 512, 1, 2, 0),
    (2, 9, 64, 64, 3, 2, 1),
    (1024, 70, 64, 64, 3, 1, 1),  # 128x64 tiles
    (512, 64, 128, 256, 3, 1, 1),  # 128x128 tiles
    (600, 64, 128, 256, 3, 2, 1),  # 128x128, strided, ragged last M tile
]


def _rel(a, b):
    return (a.float() - b.float()).norm().item() / (b.float().norm().item() + 1e-12)


@pytest.mark.parametrize("B,L,Cin,Cout,K,s,p", CASES)
def test_conv1d_nlc_forward_backward(B, L, Cin, Cout, K, s, p):
    from crossscale_ecg.ops.conv_mc import conv1d_nlc
    torch.manual_seed(0)
    x = torch.randn(B, L, Cin, device=DEV).bfloat16().requires_grad_(True)
    w = (torch.randn(Cout, Cin, K, device=DEV) / (Cin * K) ** 0.5).requires_grad_(True)
    b = torch.randn(Cout, device=DEV).requires_grad_(True)
    y = conv1d_nlc(x, w, b, s, p)
    # fp32 reference on the same bf16-rounded inputs
    xr = x.detach().float().transpose(1, 2).requires_grad_(True)
    wr = w.detach().bfloat16().float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.conv1d(xr, wr, br, stride=s, padding=p)
    assert y.shape == (B, yr.shape[2], Cout)
    assert _rel(y.transpose(1, 2), yr) < 1e-2
    g = torch.randn_like(yr)
    yr.backward(g)
    y.backward(g.transpose(1, 2).bfloat16())
    torch.cuda.synchronize()
    assert _rel(x.grad.transpose(1, 2), xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 1e-2


STRIDED = [c for c in CASES if c[5] > 1]


@pytest.mark.parametrize("B,L,Cin,Cout,K,s,p", STRIDED)
def test_strided_dgrad_dma_equals_register_loop(B, L, Cin, Cout, K, s, p):
    """The phase-decomposed strided data-grad on the LDS-DMA loop (default) and on the register-staged loop compute
    the same MFMA sums in the same order: bitwise-equal input gradients (and both match fp32, test above)."""
    from crossscale_ecg.ops.conv_mc import conv1d_nlc, set_dma_dilated, set_tap_s2
    torch.manual_seed(1)
    x0 = torch.randn(B, L, Cin, device=DEV).bfloat16()
    w = torch.randn(Cout, Cin, K, device=DEV) / (Cin * K) ** 0.5
    grads = []
    prev_s2 = set_tap_s2(False)  # the phase-decomposed one-tap kernels (the tap-shared form: test below)
    for on in (True, False):
        prev = set_dma_dilated(on)
        try:
            x = x0.clone().requires_grad_(True)
            y = conv1d_nlc(x, w, None, s, p)
            g = torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(7)).bfloat16()
            y.backward(g)
            torch.cuda.synchronize()
            grads.append(x.grad.clone())
        finally:
            set_dma_dilated(prev)
    set_tap_s2(prev_s2)
    assert torch.equal(grads[0], grads[1])


S2_CASES = [c for c in STRIDED if c[4] == 3 and c[5] == 2 and c[6] == 1] + [
    (1024, 125, 64, 128, 3, 2, 1),  # ResNet layer-2 first conv at B=1024 (dgrad: 64 output channels, odd L)
    (1024, 32, 256, 512, 3, 2, 1),  # layer-4 first conv (dgrad: 256 output channels, 4 chunks)
]


@pytest.mark.parametrize("B,L,Cin,Cout,K,s,p", S2_CASES)
def test_strided_dgrad_tap_shared(B, L, Cin, Cout, K, s, p):
    """The tap-shared strided data-grad (one staged dz image per 128 i-rows read by both output phases: tap 1 for
    even outputs, taps 0 / 2 for odd ones) against an fp64 transposed conv of the same bf16 operands, its BatchNorm
    partial rows are one per 128 i-rows, and it agrees with the phase-decomposed one-tap kernels to bf16 rounding."""
    from crossscale_ecg.ops import conv_mc
    torch.manual_seed(3)
    Lo = conv_mc.out_len(L, K, s, p)
    dy = torch.randn(B, Lo, Cout, device=DEV).bfloat16()
    wd = (torch.randn(Cin, K, Cout, device=DEV) / (Cout * K) ** 0.5).bfloat16()  # flipped [Cin][K][Cout] layout
    assert conv_mc.stat_rows(B, Lo, Cout, L, Cin, K, 1, K - 1 - p, s) == (B * Lo + 127) // 128
    dx = conv_mc.fwd_raw(dy, wd, None, 1, K - 1 - p, L, in_dil=s)
    prev = conv_mc.set_tap_s2(False)
    try:
        dx1 = conv_mc.fwd_raw(dy, wd, None, 1, K - 1 - p, L, in_dil=s)
    finally:
        conv_mc.set_tap_s2(prev)
    torch.cuda.synchronize()
    # reference: dx = conv_transpose(dy, W) with W [Cout][Cin][K] = the un-flipped forward weight
    w_fwd = wd.double().flip(1).permute(2, 0, 1)  # [Cout][Cin][K]
    ref = F.conv_transpose1d(dy.double().transpose(1, 2), w_fwd, None, stride=s, padding=p,
                             output_padding=L - ((Lo - 1) * s - 2 * p + K))
    got = dx.double().transpose(1, 2)
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    assert _rel(got, ref) < 4e-3
    assert _rel(dx.double(), dx1.double()) < 4e-3


BIG_CASES = [  # shapes that select the 256-row DMA tiles once the big-tile family is enabled
    (2048, 64, 128, 256, 3, 1, 1),  # 256x256
    (2100, 63, 128, 128, 3, 1, 1),  # 256x128, ragged last M tile
    (1030, 128, 64, 512, 3, 1, 1),  # 256x256 (2 N tiles), ragged; dgrad on 256x64 -> 128-row tiles
    (64, 32, 256, 256, 3, 1, 1),  # 256x256 weight-grad (family 2)
]


@pytest.mark.parametrize("B,L,Cin,Cout,K,s,p", BIG_CASES)
def test_conv1d_nlc_big_tiles(B, L, Cin, Cout, K, s, p):
    from crossscale_ecg.ops.conv_mc import set_tile_family
    prev = set_tile_family(2)
    try:
        test_conv1d_nlc_forward_backward(B, L, Cin, Cout, K, s, p)
    finally:
        set_tile_family(prev)


TS_CASES = [  # stride-1 3-tap shapes of the tap-shared weight gradient: chunks spanning samples, ragged last chunk
    (3, 37, 64, 128),
    (5, 8, 128, 64),  # L = 8: a sample boundary in every 8-row group
    (2, 16, 512, 512),
    (1024, 125, 64, 64),
    (256, 32, 256, 256),
]


@pytest.mark.parametrize("B,L,Cin,Cout", TS_CASES)
def test_wgrad_tap_shared_matches_fp64(B, L, Cin, Cout):
    """Weight gradient of stride-1 3-tap convs - the tap-shared kernel (one 64x64x3 block per workgroup, taps 0/2
    masked at sample boundaries; selected up to 64 channels by default) or the one-tap kernels - is an fp32 sum
    of exact bf16 products: within 1e-4 relative of an fp64 reference on the same bf16 inputs."""
    from crossscale_ecg.ops import conv_mc
    lib = conv_mc._lib_k()
    ts = lib.ecg_conv1d_nlc_wgrad_splits(B, L, Cin, L, Cout, 3, 1, 1) > 0
    assert ts == (max(Cin, Cout) <= 64)
    torch.manual_seed(3)
    x = torch.randn(B, L, Cin, device=DEV).bfloat16()
    dy = torch.randn(B, L, Cout, device=DEV).bfloat16()
    dw = conv_mc.wgrad_raw(dy, x, 3, 1, 1)  # [Cout][Cin][K] or [Cout][K][Cin] per wgrad_raw's contract
    xr = x.double().transpose(1, 2)
    ref = torch.nn.grad.conv1d_weight(xr, (Cout, Cin, 3), dy.double().transpose(1, 2), stride=1, padding=1)
    got = dw.double()
    if got.shape != ref.shape:
        got = got.permute(0, 2, 1)
    torch.cuda.synchronize()
    assert got.shape == ref.shape
    assert (got - ref).norm().item() / ref.norm().item() < 1e-4


def _grads(m, x, y, amp=False):
    m.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        F.cross_entropy(m(x), y).backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}


def test_resnet1d_hip_backend_matches_torch():
    """The hip backend (bf16 NLC MFMA convs) vs the fp32 torch model.  A random-init deep net in train-mode BN
    amplifies bf16 rounding (torch's own bf16 autocast is ~30% off fp32 in the early-layer grads at B=8), so
    the bound is relative to the autocast error of the same batch, plus an absolute cap."""
    from crossscale_ecg.models.resnet1d import resnet1d18
    torch.manual_seed(0)
    m = resnet1d18(backend="torch").to(DEV)
    x = torch.randn(16, 1, 500, device=DEV)
    y = torch.randint(0, 2, (16,), device=DEV)
    m.eval()
    with torch.no_grad():
        a = m(x)
        m.backend = "hip"
        b = m(x)
    assert _rel(b, a) < 5e-2
    m.train()
    m.backend = "torch"
    g32 = _grads(m, x, y)
    gam = _grads(m, x, y, amp=True)
    m.backend = "hip"
    ghp = _grads(m, x, y)
    for n in g32:
        e_amp, e_hip = _rel(gam[n], g32[n]), _rel(ghp[n], g32[n])
        assert e_hip < 1.5 * e_amp + 0.05 and e_hip < 0.6, (n, e_hip, e_amp)


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("B,L,C", [(1024, 125, 64), (1024, 63, 128), (700, 125, 64)])
def test_conv1d_nlc_stats_multi_tile(mode, B, L, C):
    """BatchNorm-statistics epilogue (the ResNet plan's CONV_FWD) on every forward mode: the stored outputs are the
    same bits whichever kernel runs (multi-tile workgroups compute each tile exactly like one-tile workgroups), and
    the partial rows sum to the fp64 statistics of those stored bf16 values."""
    from crossscale_ecg.ops import conv_mc
    torch.manual_seed(1)
    x = torch.randn(B, L, C, device="cuda").bfloat16()
    w = (torch.randn(C, 3, C, device="cuda") * 0.05).bfloat16()
    prev = conv_mc.set_multi_tile(0)
    prev64 = conv_mc.set_tap64(False)  # the 64-channel shapes go to the persistent tap kernel by default
    try:
        y0, _ = conv_mc.fwd_stats_raw(x, w, 1, 1, L)
        conv_mc.set_multi_tile(mode)
        y, stats = conv_mc.fwd_stats_raw(x, w, 1, 1, L)
        torch.cuda.synchronize()
    finally:
        conv_mc.set_multi_tile(prev)
        conv_mc.set_tap64(prev64)
    assert torch.equal(y, y0)
    if mode == 1 and C == 64 or mode == 2:
        assert stats.shape[1] < (B * L + 127) // 128  # the multi-tile kernel ran (fewer partial rows than tiles)
    yd = y.double().reshape(-1, C)
    s1, s2 = stats.double().sum(1)
    torch.testing.assert_close(s1, yd.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(s2, (yd * yd).sum(0), rtol=1e-5, atol=1e-3)


TAP_CASES = [  # stride-1 pad-1 3-tap convs on the tap-shared 256-row kernel: sample boundaries inside fragments,
    (3, 37, 64, 128),  # ragged last M tile (111 rows), one 64-channel chunk
    (5, 8, 128, 128),  # L = 8: boundaries every 8 rows
    (7, 2, 128, 256),  # L = 2: every row is a boundary row for one of the outer taps
    (300, 63, 128, 128),  # the ResNet layer-2 shape, 74 M tiles, ragged last tile
    (33, 16, 512, 512),  # 8 chunks x 3 taps, 4 column blocks
    (40, 125, 64, 64),  # 64-column tiles (mode 2)
]


@pytest.mark.parametrize("B,L,Cin,Cout", TAP_CASES)
def test_tap_shared_forward_matches_fp64(B, L, Cin, Cout):
    """The tap-shared kernel (A' image staged once per chunk, taps read at row offsets 0/1/2, outer taps masked at
    sample boundaries) against an fp64 conv of the same bf16 inputs, plus its BatchNorm partial rows against the
    statistics of its own stored outputs."""
    from crossscale_ecg.ops import conv_mc
    prev = conv_mc.set_tap_shared(2)
    prev64 = conv_mc.set_tap64(False)
    try:
        torch.manual_seed(11)
        x = torch.randn(B, L, Cin, device=DEV).bfloat16()
        w = (torch.randn(Cout, 3, Cin, device=DEV) / (3 * Cin) ** 0.5).bfloat16()
        y = conv_mc.fwd_raw(x, w, None, 1, 1, L)
        ys, stats = conv_mc.fwd_stats_raw(x, w, 1, 1, L)
        torch.cuda.synchronize()
        assert stats.shape[1] == (B * L + 255) // 256  # one partial row per 256-row tile
    finally:
        conv_mc.set_tap_shared(prev)
        conv_mc.set_tap64(prev64)
    ref = F.conv1d(x.double().transpose(1, 2), w.double().permute(0, 2, 1), None, stride=1, padding=1)
    got = y.double().transpose(1, 2)
    assert (got - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    assert _rel(got, ref) < 4e-3
    assert torch.equal(y, ys)
    yf = ys.float().reshape(-1, Cout)
    assert torch.allclose(stats[0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-2)
    assert torch.allclose(stats[1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-2)


TAP64_CASES = [  # C_in == C_out == 64 stride-1 3-tap convs on the persistent 64-channel kernel
    (1024, 125, 1.0),  # the ResNet layer-1 shape: 1000 tiles over 512 workgroups
    (3, 37, 1.0),  # ragged last tile (111 rows), one workgroup
    (7, 2, 1.0),  # L = 2: every row is a sample boundary for an outer tap
    (700, 125, 1.0),  # 684 tiles: some workgroups walk one tile, some two
    (64, 125, 0.0),  # zero activations: exactly zero outputs and statistics
]


@pytest.mark.parametrize("B,L,scale", TAP64_CASES)
def test_tap64_forward_matches_fp64(B, L, scale):
    """The persistent 64-channel tap kernel (weights resident in LDS, each workgroup walking M tiles with the next
    tile's A' image landing under the current tile's MFMAs and epilogue) against an fp64 conv of the same bf16
    inputs; its per-workgroup BatchNorm partial rows against the statistics of its own stored outputs; the one-tap
    kernels' outputs agree to bf16 rounding."""
    from crossscale_ecg.ops import conv_mc
    torch.manual_seed(5)
    x = (torch.randn(B, L, 64, device=DEV) * scale).bfloat16()
    w = (torch.randn(64, 3, 64, device=DEV) / 192 ** 0.5).bfloat16()
    prev = conv_mc.set_tap64(True)
    try:
        y = conv_mc.fwd_raw(x, w, None, 1, 1, L)
        ys, stats = conv_mc.fwd_stats_raw(x, w, 1, 1, L)
        conv_mc.set_tap64(False)
        y1 = conv_mc.fwd_raw(x, w, None, 1, 1, L)
        torch.cuda.synchronize()
    finally:
        conv_mc.set_tap64(prev)
    tiles = (B * L + 127) // 128
    assert stats.shape[1] == min(tiles, 2 * torch.cuda.get_device_properties(0).multi_processor_count)
    assert torch.equal(y, ys)
    ref = F.conv1d(x.double().transpose(1, 2), w.double().permute(0, 2, 1), None, stride=1, padding=1)
    got = y.double().transpose(1, 2)
    if scale == 0.0:
        assert not y.abs().any() and not stats.abs().any()
        return
    assert (got - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    assert _rel(got, ref) < 4e-3
    assert _rel(y.double(), y1.double()) < 4e-3
    yf = ys.double().reshape(-1, 64)
    torch.testing.assert_close(stats[0].double().sum(0), yf.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(stats[1].double().sum(0), (yf * yf).sum(0), rtol=1e-5, atol=1e-3)


PREACT_CASES = [  # stride-1 3-tap convs of the ResNet stages: the persistent 64-channel kernel, the 128-column tap kernel
    (1024, 125, 64, 64),  # layer 1 at B=1024: 1000 tiles over 512 persistent workgroups (one or two each)
    (3, 37, 64, 64),  # one ragged 64-channel tile
    (64, 63, 128, 128),  # layer 2, ragged last tile
    (40, 32, 256, 256),  # layer 3: 4 chunks, 2 column blocks (only nt == 0 stores the activated rows)
    (33, 16, 512, 512),  # layer 4: 8 chunks, 4 column blocks
    (3, 5, 128, 256),  # one tile, most image rows outside the tensor
]


@pytest.mark.parametrize("B,L,Cin,Cout", PREACT_CASES)
def test_tap_pre_activation_matches_fp64(B, L, Cin, Cout):
    """Input pre-activation (BatchNorm scale / shift + ReLU applied to the tap-shared kernel's staged A' image): the
    activated operand it stores equals relu(z * scale + shift) to bf16 rounding, the conv equals an fp64 conv of that
    stored operand, and the plain tap kernel on the stored operand gives bitwise the same output."""
    from crossscale_ecg.ops import conv_mc
    torch.manual_seed(9)
    z = torch.randn(B, L, Cin, device=DEV).bfloat16()
    w = (torch.randn(Cout, 3, Cin, device=DEV) / (3 * Cin) ** 0.5).bfloat16()
    sc = torch.rand(Cin, device=DEV) + 0.5
    sh = torch.randn(Cin, device=DEV) * 0.5
    assert conv_mc.pre_act_ok(B, L, Cin, Cout)
    y, act = conv_mc.fwd_pre_act_raw(z, sc, sh, w)
    torch.cuda.synchronize()
    want = torch.relu(z.double() * sc.double() + sh.double())
    assert (act.double() - want).abs().max().item() <= 8e-3 * want.abs().max().item()
    assert _rel(act.double(), want) < 4e-3
    ref = F.conv1d(act.double().transpose(1, 2), w.double().permute(0, 2, 1), None, stride=1, padding=1)
    got = y.double().transpose(1, 2)
    assert (got - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    assert _rel(got, ref) < 4e-3
    assert torch.equal(conv_mc.fwd_raw(act, w, None, 1, 1, L), y)
