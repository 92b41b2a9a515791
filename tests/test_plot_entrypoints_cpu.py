"""The reference-named plot entry points (plot_locality.py, plot_all_results.py, plot_part2.py, plot_part3.py -
Module_1/2/3's plot scripts) on the committed round-6 module CSVs: every figure the reference script draws is
written, plus the merged ``part1_all_results.csv`` with the amortised-shard columns when the shard-prep JSON
exists."""
import glob
import json
import os
import shutil
import subprocess
import sys

import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODULES = os.path.join(ROOT, "profiles", "r6", "modules")


def _run(script, d, *extra):
    out = subprocess.run([sys.executable, os.path.join(ROOT, script), "--results-dir", str(d), *extra],
                         capture_output=True, text=True, cwd=str(d))
    assert out.returncode == 0, out.stderr[-2000:]
    return out.stdout


def test_reference_plot_scripts(tmp_path):
    for f in glob.glob(os.path.join(MODULES, "*.csv")):
        shutil.copy(f, tmp_path)
    # a shard-prep metrics file (shard_prep.py's JSON keys) so the A4 amortised columns are computed
    json.dump({"total_time_s": 12.0, "total_windows": 200000}, open(tmp_path / "shard_prep_metrics.json", "w"))
    _run("plot_locality.py", tmp_path, "--batch", "256")
    assert (tmp_path / "throughput_vs_batch.png").exists() and (tmp_path / "time_breakdown_stacked.png").exists()
    _run("plot_all_results.py", tmp_path)
    for f in ("part1_all_results.csv", "throughput_comparison_A0_A4.png", "time_breakdown_batch512_A0_A4.png"):
        assert (tmp_path / f).exists(), f
    merged = pd.read_csv(tmp_path / "part1_all_results.csv")
    a4 = merged[merged["config"] == "A4_LABL"]
    assert len(a4) and a4["effective_samples_per_s"].notna().all()
    assert (a4["effective_samples_per_s"] < a4["samples_per_s"]).all()  # the amortised prep only costs
    _run("plot_part2.py", tmp_path)
    assert (tmp_path / "part2_hip_speedup.png").exists() and (tmp_path / "part2_openmp_speedup.png").exists()
    _run("plot_part3.py", tmp_path)
    for f in ("part3_throughput_vs_world.png", "part3_step_breakdown_grouped.png", "fedavg_node_scaling.png"):
        assert (tmp_path / f).exists(), f
