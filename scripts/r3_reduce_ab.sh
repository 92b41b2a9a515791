#!/bin/bash
# Round-3 late session: TinyECG bench cross-check, capped/auto-wide weight-gradient reduce correctness + A/B.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 500 --warmup 100 --no-extras > gpurun_out/b500x.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras > gpurun_out/b20x.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*, "gpu_ms_per_step": [0-9.]*' gpurun_out/b500x.log gpurun_out/b20x.log
ECG_REDUCE_GRID=64 ECG_REDUCE_WIDE=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_resnet_engine_gpu.py -k "grads" > gpurun_out/reduce_knob_tests.log 2>&1 || { tail -30 gpurun_out/reduce_knob_tests.log; exit 1; }
tail -3 gpurun_out/reduce_knob_tests.log
bash scripts/ab_resnet_cfgs.sh 3 "base|X=0" "wide2|ECG_REDUCE_WIDE=2" "grid128|ECG_REDUCE_GRID=128" "grid512|ECG_REDUCE_GRID=512"
