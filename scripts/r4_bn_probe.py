#!/usr/bin/env python3
"""Isolated timing of the ResNet engine's memory-bound BatchNorm passes at the B=1024 stage shapes: BN_ACT (forward
BN + ReLU, modes 0/1/2) and BN_BWD_APPLY (BN backward apply, plain and with the downsample branch), run through the
plan executor (ecg_plan_run) as single ops, against a torch bf16 copy of the same bytes.  One JSON line per shape.

    python scripts/r4_bn_probe.py [reps=50]
"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import crossscale_ecg  # noqa: E402,F401
from crossscale_ecg.ops import _lib  # noqa: E402
from crossscale_ecg.ops.resnet_engine import OP, OP_WORDS, _bind  # noqa: E402

SHAPES = [("l1", 1024 * 125, 64), ("l2", 1024 * 63, 128), ("l3", 1024 * 32, 256), ("l4", 1024 * 16, 512)]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    lib = _lib.kernels()
    _bind(lib)
    dev = torch.device("cuda:0")
    strm = _lib.stream_ptr(dev)
    P = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    for name, R, C in SHAPES:
        bf = lambda: torch.randn(R, C, device=dev).bfloat16()  # noqa: E731
        vec = lambda: torch.rand(C, device=dev) + 0.5  # noqa: E731
        z, res, zd, gy, out, out_d = bf(), bf(), bf(), bf(), bf(), bf()
        sc, sh, scd, shd, mu, rs, c1, c2, c2d = (vec() for _ in range(9))

        def run(words):
            ops = torch.zeros(1, OP_WORDS, dtype=torch.int64)
            ops[0, :len(words)] = torch.tensor(words, dtype=torch.int64)
            bad = ctypes.c_int(-1)

            def go():
                _lib.check(lib.ecg_plan_run(ops.data_ptr(), 1, ctypes.byref(bad), strm), "ecg_plan_run")
            return go

        mb = R * C * 2 / 1e6
        rec = {"shape": name, "R": R, "C": C, "tensor_mb": round(mb, 1)}
        cases = {
            "act0": (run([OP["BN_ACT"], 0, P(z), P(sc), P(sh), 0, 0, 0, P(out), R, C]), 2),
            "act1": (run([OP["BN_ACT"], 1, P(z), P(sc), P(sh), P(res), 0, 0, P(out), R, C]), 3),
            "act2": (run([OP["BN_ACT"], 2, P(z), P(sc), P(sh), P(zd), P(scd), P(shd), P(out), R, C]), 3),
            "apply": (run([OP["BN_BWD_APPLY"], 0, P(gy), 0, P(z), P(mu), P(rs), P(sc), P(c1), P(c2), P(out),
                           0, 0, 0, 0, 0, 0, R, C]), 3),
            "apply_ds": (run([OP["BN_BWD_APPLY"], 1, P(gy), 0, P(z), P(mu), P(rs), P(sc), P(c1), P(c2), P(out),
                              P(zd), P(mu), P(rs), P(scd), P(c2d), P(out_d), R, C]), 5),
            "copy": (lambda: out.copy_(z), 2),
        }
        for k, (fn, ntens) in cases.items():
            us = timeit(fn, reps)
            rec[k + "_us"] = round(us, 2)
            rec[k + "_tbs"] = round(ntens * mb / us, 2)  # MB/us = TB/s
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
