import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_addoption(parser):
    parser.addoption("--hip-serialize", action="store_true",
                     help="debug mode: AMD_SERIALIZE_KERNEL=3 + HIP_LAUNCH_BLOCKING=1 (every launch synchronous, so "
                          "a faulting kernel is reported at its own launch)")


def pytest_configure(config):
    if config.getoption("--hip-serialize", default=False):
        os.environ["AMD_SERIALIZE_KERNEL"] = "3"
        os.environ["HIP_LAUNCH_BLOCKING"] = "1"
        os.environ["AMD_SERIALIZE_COPY"] = "3"
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the HIP kernels")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")
    # Build (incrementally, seconds when cached) the native libraries so CPU tests can load the
    # C++ kernels and GPU tests never silently run without the HIP library.
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    try:
        import build as native_build
        native_build.build_all(force=False, jobs=min(8, os.cpu_count() or 1), verbose=False)
    except Exception as e:  # pragma: no cover - toolchain missing
        print(f"[conftest] native build failed: {e}")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def tmpdir_path(tmp_path):
    return str(tmp_path)
