"""scripts/trace_module1_b128.py parse: per-configuration medians of the roctx compute ranges (wall, GPU kernel busy,
kernels, host time in launch calls, host gaps between HIP calls) from synthetic rocprofv3 marker / kernel / HIP API
trace CSVs; and the roctx library order (rocprofv3 records the rocprofiler-sdk library's markers)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _write(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_trace_parse_splits_gpu_and_host_time(tmp_path):
    hdr = ["Domain", "Function", "Process_Id", "Thread_Id", "Correlation_Id", "Start_Timestamp", "End_Timestamp"]
    markers, hip, kern = [], [], []
    for i in range(4):  # A0 ranges: 100 us wall; A3 ranges: 150 us wall; same two 20 us kernels in each
        for name, t0, wall in (("A0/compute", i * 1_000_000, 100_000), ("A3/compute", i * 1_000_000 + 500_000, 150_000)):
            markers.append(["MARKER", name, 1, 7, 0, t0, t0 + wall])
            hip.append(["HIP", "hipLaunchKernel", 1, 7, 0, t0 + 1_000, t0 + 6_000])
            hip.append(["HIP", "hipLaunchKernel", 1, 7, 0, t0 + 46_000 if wall == 100_000 else t0 + 96_000,
                        t0 + 51_000 if wall == 100_000 else t0 + 101_000])
            kern.append([t0 + 10_000, t0 + 30_000, "k1"])
            kern.append([t0 + 60_000, t0 + 80_000, "k2"])
    _write(tmp_path / "t_marker_api_trace.csv", hdr, markers)
    _write(tmp_path / "t_hip_api_trace.csv", hdr, hip)
    _write(tmp_path / "t_kernel_trace.csv", ["Start_Timestamp", "End_Timestamp", "Kernel_Name"], kern)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_module1_b128.py"), "parse",
                          str(tmp_path)], capture_output=True, text=True, check=True).stdout
    lines = {ln.split(":")[0].strip(): ln for ln in out.splitlines() if ln.strip().startswith(("A0:", "A3:"))}
    assert "wall    100.0" in lines["A0"] and "wall    150.0" in lines["A3"], out
    assert "gpu    40.0" in lines["A0"] and "gpu    40.0" in lines["A3"], out   # same GPU work
    assert "launch    10.0" in lines["A0"] and "launch    10.0" in lines["A3"], out
    assert "gaps    40.0" in lines["A0"] and "gaps    90.0" in lines["A3"], out   # the extra wall is host gaps


def test_roctx_prefers_the_rocprofiler_sdk_library():
    import crossscale_ecg  # noqa: F401
    from crossscale_ecg.utils import profiling
    sdk = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib", "librocprofiler-sdk-roctx.so")
    lib = profiling._lib()
    if os.path.exists(sdk):
        assert lib is not None and lib._name == sdk
    with profiling.range("x"):  # a no-op range works with or without a library
        pass
