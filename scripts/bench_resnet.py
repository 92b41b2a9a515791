#!/usr/bin/env python3
"""ResNet1D-34 stress benchmark: per-layer MFMA conv vs MIOpen, then training throughput of the native step
engine vs PyTorch (MIOpen, bf16 autocast) and the autograd ``hip`` backend, over batch sizes."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.resnet import engine_throughput, layer_table, train_throughput  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="256,1024,4096")
    ap.add_argument("--layers", action="store_true")
    ap.add_argument("--backends", default="engine,torch,hip")
    a = ap.parse_args()
    if a.layers:
        for r in layer_table():
            print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    for B in [int(b) for b in a.batches.split(",")]:
        for be in a.backends.split(","):
            v = engine_throughput(B=B) if be == "engine" else train_throughput(be, B=B)
            print(json.dumps({"model": "resnet1d34", "backend": be, "batch": B, "L": 500,
                              "train_samples_per_s": round(v, 1)}), flush=True)
