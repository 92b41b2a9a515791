"""C++ native pieces that run without a GPU: CPU conv1d kernel (reference C ABI) and the IO prefetcher."""
import ctypes

import numpy as np
import pytest
import torch

import crossscale_ecg  # noqa: F401
from crossscale_ecg.ops import _lib
from crossscale_ecg.ops.conv1d import run_omp_conv, conv1d_valid, conv1d_valid_reference


@pytest.mark.parametrize("K", [1, 3, 5, 7, 8, 17, 32])
@pytest.mark.parametrize("isa", [0, 1, 2])
def test_cpu_conv_matches_numpy(K, isa):
    lib = _lib.cpu_lib()
    got_isa = lib.conv1d_cpu_set_isa(isa)
    try:
        rng = np.random.default_rng(K)
        x = rng.normal(size=(37, 500)).astype(np.float32)
        w = rng.normal(size=(K,)).astype(np.float32)
        y = run_omp_conv(x, w, nthreads=3)
        ref = conv1d_valid_reference(x, w)
        assert y.shape == (37, 500 - K + 1)
        assert np.abs(y - ref).max() < 1e-4
        assert got_isa <= isa
    finally:
        lib.conv1d_cpu_set_isa(-1)


def test_cpu_conv_isas_bitwise_identical():
    lib = _lib.cpu_lib()
    x = np.random.default_rng(0).normal(size=(8, 300)).astype(np.float32)
    w = np.random.default_rng(1).normal(size=(7,)).astype(np.float32)
    outs = []
    for isa in (0, 1, 2):
        lib.conv1d_cpu_set_isa(isa)
        outs.append(run_omp_conv(x, w, 2).copy())
    lib.conv1d_cpu_set_isa(-1)
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])


def test_reference_c_abi_symbol():
    lib = _lib.cpu_lib()
    fn = lib.conv1d_batch_omp_simd  # exact exported name of Module_2/conv1d_openmp_simd.c
    x = np.ones((2, 10), np.float32)
    w = np.ones(3, np.float32)
    y = np.zeros((2, 8), np.float32)
    fp = ctypes.POINTER(ctypes.c_float)
    fn(x.ctypes.data_as(fp), w.ctypes.data_as(fp), y.ctypes.data_as(fp), 2, 10, 3, 1)
    assert np.all(y == 3)


def test_conv1d_valid_cpu_and_torch_backends_agree():
    x = torch.randn(16, 1, 100)
    w = torch.randn(5)
    a = conv1d_valid(x, w, backend="cpu")
    b = conv1d_valid(x, w, backend="torch")
    assert a.shape == b.shape == (16, 1, 96)
    assert torch.allclose(a, b, atol=1e-5)


def _shards(tmp_path, n=500, L=40, size=128):
    from crossscale_ecg.data.shards import write_shards
    data = np.random.default_rng(3).normal(2.0, 3.0, size=(n, L)).astype(np.float32)
    return data, write_shards(data, str(tmp_path), shard_size=size)


def test_mapped_shard(tmp_path):
    from crossscale_ecg.ops.native_io import MappedShard
    data, paths = _shards(tmp_path)
    with MappedShard(paths[1]) as m:
        assert (m.N, m.L) == (128, 40)
        assert np.array_equal(m.array, data[128:256])


@pytest.mark.parametrize("normalize", [False, True])
def test_prefetcher_order_normalize_eof(tmp_path, normalize):
    from crossscale_ecg.ops.native_io import NativePrefetcher
    data, paths = _shards(tmp_path)
    pf = NativePrefetcher(paths, batch_size=50, num_slots=3, normalize=normalize, pinned=False)
    pf.start()
    got, sizes = [], []
    while True:
        r = pf.next_batch_cpu()
        if r is None:
            break
        slot, view, ms = r
        assert view.shape[1:] == (1, 40) and ms >= 0
        got.append(view[:, 0].clone().numpy())
        sizes.append(view.shape[0])
        pf.recycle(slot)
    pf.close()
    allx = np.concatenate(got)
    ref = data.astype(np.float64)
    if normalize:
        ref = (ref - ref.mean(1, keepdims=True)) / (ref.std(1, keepdims=True) + 1e-8)
    assert allx.shape == data.shape
    assert np.abs(allx - ref).max() < 1e-5
    # batches never span shards (reference semantics): 128 = 50 + 50 + 28
    assert sizes[:3] == [50, 50, 28]


def test_prefetcher_loop_mode_and_shutdown(tmp_path):
    from crossscale_ecg.ops.native_io import NativePrefetcher
    _data, paths = _shards(tmp_path, n=100, size=100)
    pf = NativePrefetcher(paths, batch_size=40, num_slots=2, normalize=False, pinned=False, loop=True)
    pf.start()
    for _ in range(10):  # more than one epoch worth of batches
        slot, view, _ = pf.next_batch_cpu()
        pf.recycle(slot)
    pf.close()  # joins the producer thread


def test_labl_compat_api(tmp_path):
    """Reference LABL API names (labl_loader(EXPERIMENTAL).py): open_shard yields (mm, base, N, L) that
    np.frombuffer reads exactly like the reference; the prefetcher keeps its constructor and methods."""
    import labl_loader
    data, paths = _shards(tmp_path)
    reader = labl_loader.LABLShardedReader(paths)
    with reader.open_shard(paths[2]) as (mm, base, N, L):
        assert (base, N, L) == (16, 128, 40)
        w5 = np.frombuffer(mm, dtype=np.float32, count=L, offset=base + 5 * L * 4)
        assert np.array_equal(w5, data[256 + 5])
    ring = labl_loader.PinnedRing(3, (8, 1, 40))
    assert len(ring.slots) == 3 and ring.q_free.qsize() == 3 and ring.q_full.empty()
    pf = labl_loader.LABLPrefetcher(reader, batch_size=64, num_slots=2, normalize=False, pinned=False)
    assert (pf.L, pf.B) == (40, 64)
    pf.start()
    got = [b[:, 0].clone().numpy() for b, ms in pf]
    pf.close()
    assert np.array_equal(np.concatenate(got), data)


def test_labl_open_shard_view_outlives_block(tmp_path):
    import labl_loader
    data, paths = _shards(tmp_path)
    with labl_loader.LABLShardedReader(paths).open_shard(paths[0]) as (mm, base, N, L):
        w = np.frombuffer(mm, dtype=np.float32, count=N * L, offset=base)
    assert np.array_equal(w.reshape(N, L), data[:N])  # mapping stays until the last view is dropped


def test_bench_labl_cpu_glob(tmp_path):
    """A4 benchmark on the CPU device, shards given as the reference's glob string."""
    from crossscale_ecg.bench.module1 import bench_labl
    _shards(tmp_path, n=300, L=500, size=128)
    st = bench_labl(str(tmp_path / "ecg_*.bin"), 32, 3, True, "cpu")
    assert st["samples_per_s"] > 0 and st["step_ms"] > 0
