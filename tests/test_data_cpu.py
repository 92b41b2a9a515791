"""Shard format, assignment, datasets and samplers (CPU)."""
import json
import os

import numpy as np
import pytest
import torch

import crossscale_ecg  # noqa: F401
from crossscale_ecg.data import shards as S
from crossscale_ecg.data.dataset import (ShardDataset, make_dataloader, load_shards_to_gpu, make_gpu_batch_iter,
                                         DeviceIndexSampler)


def test_shard_roundtrip_and_layout(tmp_path):
    x = np.arange(12, dtype=np.float32).reshape(3, 4)
    p = str(tmp_path / "ecg_00000.bin")
    nbytes = S.write_shard(p, x)
    assert nbytes == 16 + 48 == os.path.getsize(p)
    raw = open(p, "rb").read()
    assert np.frombuffer(raw[:16], "<i8").tolist() == [3, 4]
    assert np.array_equal(np.frombuffer(raw[16:], "<f4").reshape(3, 4), x)
    assert np.array_equal(S.load_shard(p), x)
    assert np.array_equal(np.asarray(S.load_shard(p, mmap=True)), x)
    assert S.shard_header(p) == (3, 4)


def test_bad_shard_size_raises(tmp_path):
    p = str(tmp_path / "ecg_00000.bin")
    S.write_shard(p, np.zeros((2, 5), np.float32))
    with open(p, "ab") as f:
        f.write(b"\0\0\0\0")
    with pytest.raises(RuntimeError):
        S.load_shard(p)


def test_write_shards_split(tmp_path):
    w = S.make_synth_windows(100, 16, seed=1)
    paths = S.write_shards(w, str(tmp_path), shard_size=32)
    assert [os.path.basename(p) for p in paths] == [f"ecg_{i:05d}.bin" for i in range(4)]
    assert [S.shard_header(p)[0] for p in paths] == [32, 32, 32, 4]
    assert np.array_equal(np.concatenate([S.load_shard(p) for p in paths]), w)


def test_synth_windows_match_reference_generator():
    w = S.make_synth_windows(5, 7, seed=1337)
    ref = np.random.default_rng(1337).normal(0, 1, size=(5, 7)).astype(np.float32)
    assert np.array_equal(w, ref)


def test_assign_shards_evenly():
    paths = [f"ecg_{i:05d}.bin" for i in range(7)]
    a = [S.assign_shards_evenly(paths, 3, r) for r in range(3)]
    assert a[0] == ["ecg_00000.bin", "ecg_00003.bin", "ecg_00006.bin"]
    assert sorted(sum(a, [])) == sorted(paths)
    # fewer shards than ranks: wrap-around duplicates
    few = ["b", "a"]
    assert [S.assign_shards_evenly(few, 4, r) for r in range(4)] == [["a"], ["b"], ["a"], ["b"]]
    with pytest.raises(RuntimeError):
        S.assign_shards_evenly([], 2, 0)


def test_dataset_and_loader(tmp_path):
    w = S.make_synth_windows(300, 20)
    paths = S.write_shards(w, str(tmp_path), shard_size=128)
    ds = ShardDataset(paths, max_windows=250)
    assert len(ds) == 250 and ds.y.dtype == torch.long and int(ds.y.abs().sum()) == 0
    xi, yi = ds[3]
    assert xi.shape == (1, 20) and torch.equal(xi[0], torch.from_numpy(w[3]))
    dl, n = make_dataloader(paths, 64, max_windows=250, num_workers=0)
    assert n == 250 and len(dl) == 3  # drop_last
    xb, yb = next(iter(dl))
    assert xb.shape == (64, 1, 20)
    x_d, y_d = load_shards_to_gpu(paths, "cpu", max_windows=250)
    assert torch.equal(x_d, torch.from_numpy(w[:250]))


def test_gpu_batch_iter_semantics():
    x = torch.arange(10 * 3, dtype=torch.float32).view(10, 3)
    y = torch.arange(10)
    it = make_gpu_batch_iter(x, y, 4)
    seen = []
    for _ in range(2):  # one epoch = 2 batches (drop last 2)
        xb, yb = next(it)
        assert xb.shape == (4, 1, 3)
        assert torch.equal(xb[:, 0, 0] / 3, yb.float())
        seen += yb.tolist()
    assert len(set(seen)) == 8


def test_device_index_sampler_epochs():
    s = DeviceIndexSampler(10, 4, "cpu", seed=0)
    tab = torch.empty((5, 4), dtype=torch.int32)
    s.fill(tab)
    # steps 0,1 = epoch 1 ; 2,3 = epoch 2 ; 4 = epoch 3
    for e in (tab[0:2], tab[2:4]):
        assert len(set(e.reshape(-1).tolist())) == 8
    assert tab.min() >= 0 and tab.max() < 10
    with pytest.raises(ValueError):
        s.fill(torch.empty((2, 3), dtype=torch.int32))


def test_prep_cli(tmp_path):
    from crossscale_ecg.data.prep import main
    m = main(["--dataset", "synthetic", "--n-windows", "1000", "--shard_size", "300", "--win_len", "50",
              "--out-dir", str(tmp_path / "shards"), "--results-dir", str(tmp_path / "results")])
    assert m["num_shards"] == 4 and m["total_windows"] == 1000
    js = json.load(open(tmp_path / "results" / "shard_prep_metrics.json"))
    assert set(js) == {"dataset", "total_windows", "window_len", "shard_size_windows", "num_shards", "load_time_s",
                       "write_time_s", "total_time_s", "timestamp"}
    assert len(S.list_shards(str(tmp_path / "shards"))) == 4


@pytest.mark.parametrize("E", [1, 3, None])
def test_device_index_sampler_epoch_blocks(E):
    """Batched multi-epoch permutations: every epoch is a drop-last slice of a permutation of [0, N)."""
    N, B = 103, 10
    s = DeviceIndexSampler(N, B, "cpu", seed=1, epochs_per_block=E)
    spe = N // B
    tab = torch.empty((spe * 7 + 4, B), dtype=torch.int32)
    s.fill(tab[:5])
    s.fill(tab[5:])  # refills span block boundaries
    for e in range(7):
        v = tab[e * spe:(e + 1) * spe].reshape(-1).tolist()
        assert len(set(v)) == spe * B and min(v) >= 0 and max(v) < N
    assert not torch.equal(tab[:spe], tab[spe:2 * spe])
