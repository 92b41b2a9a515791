"""scripts/resnet_timeline.py parse: per-queue busy time, overlap and the main queue's idle gaps from a synthetic
rocprofv3 kernel-trace CSV (two queues, six steps; the parser reads the last four)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_timeline_parse_reports_main_queue_gaps(tmp_path):
    rows = []
    # per step (period 100 us): main queue weight_prep [0,10) conv [12,40) apply [45,60); side queue wgrad [15,50)
    for s in range(6):
        t = s * 100_000
        rows += [(t + 0, t + 10_000, 1, "weight_prep_kernel"), (t + 12_000, t + 40_000, 1, "conv_kernel"),
                 (t + 45_000, t + 60_000, 1, "bn_bwd_apply_kernel"), (t + 15_000, t + 50_000, 2, "wgrad_kernel")]
    path = tmp_path / "trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Start_Timestamp", "End_Timestamp", "Queue_Id", "Kernel_Name"])
        for r in rows:
            w.writerow(r)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "resnet_timeline.py"), "parse", str(path)],
                         capture_output=True, text=True, check=True).stdout
    # steps are delimited by the weight prep: 4 complete steps of 100 us
    assert "100.0 us/step wall" in out
    # main queue: gaps of 2 + 5 us inside each of the 4 steps and 40 us before each of the 3 next weight preps inside
    # the window: (4 * 7 + 3 * 40) / 4 = 37 us/step
    assert "main queue 1: idle between kernels 37.0 us/step" in out, out
    assert "after conv_kernel  ->  bn_bwd_apply_kernel" in out
