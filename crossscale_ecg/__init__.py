"""Importable alias for the framework package.

The framework source lives in the directory
``crossscale-ecg-a-modular-hpc-pipeline-from-locality-optimization-to-mpi-gpu-overlap_amd/``
(a name Python cannot import directly because of the dashes).  This shim points the
package search path at that directory and runs its ``__init__`` so that
``import crossscale_ecg.models.tiny_ecg`` etc. resolve to the real sources.
"""
import os as _os

_REAL_NAME = "crossscale-ecg-a-modular-hpc-pipeline-from-locality-optimization-to-mpi-gpu-overlap_amd"
_REAL_DIR = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))), _REAL_NAME)
if not _os.path.isdir(_REAL_DIR):  # pragma: no cover - broken checkout
    raise ImportError(f"crossscale_ecg: package sources not found at {_REAL_DIR}")

__path__ = [_REAL_DIR]
_init = _os.path.join(_REAL_DIR, "__init__.py")
with open(_init, "r") as _f:
    exec(compile(_f.read(), _init, "exec"))
