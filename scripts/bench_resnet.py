#!/usr/bin/env python3
"""ResNet1D-34 stress benchmark: per-layer MFMA conv vs MIOpen + training throughput (hip vs torch backend)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.resnet import layer_table, train_throughput  # noqa: E402

if __name__ == "__main__":
    rows = layer_table()
    for r in rows:
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))
    for be in ("torch", "hip"):
        for B in (256, 1024):
            print(json.dumps({"model": "resnet1d34", "backend": be, "batch": B, "L": 500,
                              "train_samples_per_s": round(train_throughput(be, B=B), 1)}), flush=True)
