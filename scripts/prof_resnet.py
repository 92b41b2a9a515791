#!/usr/bin/env python3
"""Run a few ResNet1D-34 training steps on one backend (for rocprofv3 --kernel-trace --stats)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.bench.resnet import engine_throughput, train_throughput  # noqa: E402

if __name__ == "__main__":
    be = sys.argv[1] if len(sys.argv) > 1 else "engine"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    v = engine_throughput(B=B, steps=10) if be == "engine" else train_throughput(be, B=B, steps=10)
    print(be, B, v)
