from .tiny_ecg import TinyECG, param_layout, num_params  # noqa: F401

Tiny1D = TinyECG  # Module_1/bench_locality.py:8-21 declares the same network as ``Tiny1D``


def build_model(name: str, num_classes: int = 2, **kw):
    name = name.lower()
    if name in ("tiny_ecg", "tinyecg", "tiny1d"):
        return TinyECG(num_classes=num_classes)
    if name in ("resnet1d34", "resnet1d-34", "resnet34"):
        from .resnet1d import resnet1d34
        return resnet1d34(num_classes=num_classes, **kw)
    if name in ("resnet1d18", "resnet1d-18", "resnet18"):
        from .resnet1d import resnet1d18
        return resnet1d18(num_classes=num_classes, **kw)
    raise ValueError(f"unknown model {name!r}")
