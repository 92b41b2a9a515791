"""ThreadSanitizer run of the C++ prefetch ring, host-only: builds csrc/io/shard_io.cpp with
-fsanitize=thread into a small harness and fails on any reported race."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_shard(path, N, L):
    with open(path, "wb") as f:
        np.array([N, L], dtype=np.int64).tofile(f)
        np.repeat(np.arange(N, dtype=np.float32)[:, None], L, axis=1).tofile(f)


def _cxx():
    """ROCm's clang (current compiler-rt TSan). GCC 11's libtsan reports false 'double lock' races on this
    kernel (6.x, 28-bit mmap randomisation), so it is only the fallback."""
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    clang = os.path.join(rocm, "lib", "llvm", "bin", "clang++")
    return clang if os.path.exists(clang) else shutil.which("g++")


@pytest.mark.skipif(_cxx() is None, reason="needs a C++ compiler")
def test_prefetch_ring_tsan(tmp_path):
    exe = tmp_path / "tsan_prefetch"
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    cmd = [_cxx(), "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-D__HIP_PLATFORM_AMD__",
           f"-I{rocm}/include", os.path.join(ROOT, "tests", "native", "tsan_prefetch.cpp"),
           os.path.join(ROOT, "csrc", "io", "shard_io.cpp"), "-o", str(exe), f"-L{rocm}/lib", "-lamdhip64",
           f"-Wl,-rpath,{rocm}/lib", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        if "tsan" in r.stderr.lower() or "sanitize" in r.stderr.lower():
            pytest.skip("toolchain without ThreadSanitizer: " + r.stderr[-300:])
        raise AssertionError(r.stderr[-2000:])
    shard = tmp_path / "ecg_00000.bin"
    _write_shard(shard, 50, 16)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 report_signal_unsafe=0")
    r = subprocess.run([str(exe), str(shard), "50"], capture_output=True, text=True, env=env, timeout=120)
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr[-2000:])
    assert "tsan harness ok" in r.stdout
