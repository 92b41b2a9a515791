"""API-compatible module path of the reference ``tiny_ecg_model`` (Module_3/tiny_ecg_model.py).

``from tiny_ecg_model import TinyECG`` gives the framework's TinyECG (same architecture and state_dict
keys; adds ``flatten_parameters()`` for the fused HIP step and single-buffer FedAvg)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from crossscale_ecg.models.tiny_ecg import TinyECG, param_layout, num_params  # noqa: E402,F401

Tiny1D = TinyECG
__all__ = ["TinyECG", "Tiny1D", "param_layout", "num_params"]
