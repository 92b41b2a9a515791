"""HBM-scale GPU-resident shards (BASELINE config 5): >= 16 GiB of shard files per GPU through the native
pinned upload pipeline, verified (per-shard float64 sums + bitwise sampled rows against the files) and trained
on with one fused round.  Size: ECG_HBM_TEST_GB (default 16); skipped when the scratch disk cannot hold it."""
import os
import shutil

import pytest
import torch

import crossscale_ecg  # noqa: F401

pytestmark = pytest.mark.gpu


def test_hbm_scale_upload_and_train(tmp_path_factory):
    from crossscale_ecg.bench.hbm import run
    gb = float(os.environ.get("ECG_HBM_TEST_GB", "16"))
    d = os.environ.get("ECG_HBM_DIR") or str(tmp_path_factory.mktemp("hbm"))
    free = shutil.disk_usage(d).free / 2**30
    if free < gb * 1.2 + 2:
        pytest.skip(f"scratch disk has {free:.0f} GiB free, needs {gb * 1.2 + 2:.0f}")
    rec = run(gb, d, train=True, keep=False)
    print(rec)
    assert rec["gb_uploaded"] >= gb * 0.999
    assert rec["checksum_ok"] and rec["rows_bitwise_ok"]
    assert rec["fused_round_finite"]
    assert rec["upload_GBps"] > 1.0
