"""C ABI of the native libraries vs their ctypes bindings: every bound function's argument count equals the number of
parameters of its ``ECG_API`` / ``extern "C"`` declaration in csrc/.  A binding one argument short passes garbage
as the stream and crashes the host process only on a GPU box (round 5: fwd_ex gained ``apply``), so it is pinned
here, on the CPU."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_DECL = re.compile(r"(?:ECG_API|extern \"C\")\s+[\w\s\*]+?\b(ecg_\w+|conv1d_\w+)\s*\(([^)]*)\)\s*[{;]", re.S)


def _c_arity():
    out = {}
    srcs = glob.glob(os.path.join(ROOT, "csrc", "**", "*.hip"), recursive=True) + \
        glob.glob(os.path.join(ROOT, "csrc", "**", "*.cpp"), recursive=True)
    for path in srcs:
        text = open(path).read()
        for m in _DECL.finditer(text):
            params = m.group(2).strip()
            n = 0 if params in ("", "void") else params.count(",") + 1
            out.setdefault(m.group(1), set()).add(n)
    return out


def _bound(lib):
    return {name: fn for name, fn in vars(lib).items()
            if not name.startswith("_") and getattr(fn, "argtypes", None) is not None}


def test_ctypes_bindings_match_c_declarations():
    from crossscale_ecg.ops import _lib
    try:
        kern = _lib.kernels()
    except Exception as e:  # pragma: no cover - no native build
        pytest.skip(f"native kernels not built: {e!r}")
    from crossscale_ecg.ops import conv_mc, resnet_engine
    conv_mc._bind(kern)
    resnet_engine._bind(kern)
    libs = [kern]
    try:
        libs.append(_lib.io_lib())
    except Exception:
        pass
    arity = _c_arity()
    checked, bad = 0, []
    for lib in libs:
        for name, fn in _bound(lib).items():
            if name not in arity:
                continue
            checked += 1
            if len(fn.argtypes) not in arity[name]:
                bad.append((name, len(fn.argtypes), sorted(arity[name])))
    assert checked >= 40, checked
    assert not bad, bad
