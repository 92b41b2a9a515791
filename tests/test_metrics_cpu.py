"""Metric formulas, CSV schemas and the TinyECG parameter layout against the reference definitions
(SURVEY §4.1 / §5.5): the numbers every benchmark reports must mean what the reference's meant."""
import csv

import pytest
import torch

import crossscale_ecg  # noqa: F401
from crossscale_ecg.report.plots import effective_a4_throughput, shard_ms_per_step, EPOCHS
from crossscale_ecg.utils import csvio


def test_effective_a4_throughput_matches_reference_formula():
    # Module_1/plot_all_results.py:53-58: sps / (1 + shard_time / (EPOCHS * N / sps)), EPOCHS = 10
    sps, shard_s, n = 12_000.0, 3.5, 200_000
    ref = sps / (1 + shard_s / (EPOCHS * n / sps))
    assert EPOCHS == 10
    assert effective_a4_throughput(sps, shard_s, n) == pytest.approx(ref, rel=1e-12)
    # no preparation cost -> unchanged; amortised cost only ever lowers the throughput
    assert effective_a4_throughput(sps, 0.0, n) == pytest.approx(sps)
    assert effective_a4_throughput(sps, 100.0, n) < sps


def test_shard_ms_per_step_matches_reference_formula():
    # Module_1/plot_all_results.py:84-90: (shard_time / EPOCHS) / (N / bs) * 1e3
    assert shard_ms_per_step(3.5, 200_000, 256) == pytest.approx((3.5 / 10) / (200_000 / 256) * 1e3)


def test_part2_speedup_is_median_ratio(tmp_path):
    # Module_2/benchmark_part_2.py:92-108: medians over trials, speedup_med = torch_med / omp_med,
    # sps = B / (median_ms / 1e3); run the real CPU pair benchmark on a tiny grid point
    import statistics

    import numpy as np
    from crossscale_ecg.bench.module2 import bench_pair_cpu
    from crossscale_ecg.ops import _lib
    if not _lib.cpu_available():
        pytest.skip("libconv1d_cpu.so not built")
    row, raw = bench_pair_cpu(64, 5, np.random.default_rng(0), nthreads=2, trials=3)
    assert len(raw) == 3 and row["max_abs_err"] < 1e-4
    assert row["torch_ms_median"] == pytest.approx(statistics.median([t for t, _ in raw]))
    assert row["speedup_med"] == pytest.approx(row["torch_ms_median"] / row["omp_ms_median"])
    assert row["omp_sps"] == pytest.approx(64 / (row["omp_ms_median"] / 1e3))
    p = csvio.write_csv(str(tmp_path / "p2.csv"), [row], csvio.PART2_COLUMNS)
    with open(p) as f:
        assert next(csv.reader(f)) == csvio.PART2_COLUMNS


def test_reference_csv_schemas():
    # Module_3/part3_mpi_gpu_train.py:64-75 (BenchStats) and TRUE_FL_M3/part3_fedavg_overlap_mpi_gpu.py:41-55
    assert csvio.BENCH_COLUMNS == ["config", "world_size", "rank", "batch_size", "steps", "data_ms", "h2d_ms",
                                   "compute_ms", "step_ms", "samples_per_s"]
    # the reference RoundStats columns come first and in order; MI355X additions follow
    assert csvio.ROUND_COLUMNS[:len(csvio.ROUND_COLUMNS_REF)] == csvio.ROUND_COLUMNS_REF
    assert "comm_exposed_ms" in csvio.ROUND_COLUMNS


def test_append_results_aligns_to_existing_header(tmp_path):
    p = str(tmp_path / "r.csv")
    csvio.append_results([{"a": 1, "b": 2}], p, columns=["a", "b"])
    csvio.append_results([{"b": 4, "a": 3, "extra": 9}], p)  # extra column dropped, order from the header
    rows = csvio.read_csv(p)
    assert [r["a"] for r in rows] == ["1", "3"] and [r["b"] for r in rows] == ["2", "4"]
    assert set(rows[0]) == {"a", "b"}


def test_module1_samples_per_s_formula():
    # Module_1/bench_locality.py:73-74: samples_per_s = (samples / iters) / (step_ms / 1e3)
    samples, iters, step_ms = 256 * 100, 100, 2.5
    assert (samples / iters) / (step_ms / 1e3) == pytest.approx(102_400.0)


def test_tiny_ecg_layout_and_keys():
    from crossscale_ecg.models.tiny_ecg import TinyECG, num_params, param_layout
    m = TinyECG(num_classes=2)
    assert sum(p.numel() for p in m.parameters()) == 1458 == num_params(2)
    keys = ["net.0.weight", "net.0.bias", "net.2.weight", "net.2.bias", "head.weight", "head.bias"]
    assert list(m.state_dict().keys()) == keys
    lay = param_layout(2)
    assert list(lay.keys()) == keys
    off = 0
    for (name, (o, shape)), p in zip(lay.items(), m.parameters()):
        assert o == off and tuple(p.shape) == shape, name
        off += p.numel()
    # the flat buffer keeps state_dict round trips working
    flat = m.flatten_parameters()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    with torch.no_grad():
        flat.mul_(0.5)
    m.load_state_dict(sd)
    assert torch.allclose(m.state_dict()["net.2.weight"], sd["net.2.weight"])
