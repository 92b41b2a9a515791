"""Module-2 single-call host settings (bench/module2.py): the spin-wait flag goes through the HIP runtime torch
itself mapped (never a second, unversioned ``libamdhip64.so``), and the record is what gets written next to the CSV
(advisor r5, medium)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench import module2  # noqa: E402


def test_spin_flag_uses_torchs_hip_runtime():
    path = module2._loaded_hip_runtime()
    assert path is not None and "libamdhip64.so" in path
    assert os.path.dirname(path) == os.path.join(os.path.dirname(torch.__file__), "lib")
    rec = module2.spin_sync_flag()
    assert rec["hip_runtime"] == path
    if not torch.cuda.is_available():  # no device: the call fails and the record says so (never claims spin)
        assert rec["spin_sync"] is False


def test_pin_timing_thread_records_cpu():
    prev = os.sched_getaffinity(0)
    rec = {"pinned_cpu": None}
    try:
        module2.pin_timing_thread(rec)
        if len(prev) > 1:
            assert rec["pinned_cpu"] == min(prev) and os.sched_getaffinity(0) == {min(prev)}
    finally:
        os.sched_setaffinity(0, prev)
