"""bench.py output contract on one GPU: one JSON line with the driver's keys, whole-job value consistent with
ms_per_step, for the TinyECG headline config and the ResNet1D-34 stress config (small step counts)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def _check(rec, steps, warmup, batch):
    assert KEYS <= set(rec), KEYS - set(rec)
    assert rec["n_gpus"] == 1 and rec["steps"] == steps and rec["warmup"] == warmup
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak" and rec["dtype"] == "bf16"
    assert rec["data"] == "synthetic" and rec["unit"] == "samples/s" and rec["vs_baseline"] is None
    cfg = rec["config"]
    assert cfg["global_batch"] == batch and cfg["seq_len"] == 500 and cfg["parallelism"] == "dp1"
    # value is samples/s over the timed steps: batch * steps / (ms_per_step * steps / 1e3), up to rounding
    assert rec["value"] == pytest.approx(batch / (rec["ms_per_step"] / 1e3), rel=1e-3)


def test_bench_tiny_ecg_contract():
    rec = _bench("--steps", "100", "--warmup", "50", "--no-extras")
    _check(rec, 100, 50, 256)
    assert rec["config"]["model"].startswith("TinyECG")
    assert rec["final_avg_loss"] is not None and rec["final_avg_loss"] == rec["final_avg_loss"]


def test_bench_resnet_contract():
    rec = _bench("--model", "resnet1d34", "--batch-size", "64", "--steps", "3", "--warmup", "2", "--no-extras")
    _check(rec, 3, 2, 64)
    assert rec["config"]["model"].startswith("resnet1d34")
