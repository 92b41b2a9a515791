#!/bin/bash
# Wide weight-gradient reduce threshold A/B (ResNet1D-34 B=1024), interleaved reps.
set -u
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_resnet_engine_gpu.py -k "grads" > gpurun_out/reduce_default_tests.log 2>&1 || { tail -30 gpurun_out/reduce_default_tests.log; exit 1; }
tail -1 gpurun_out/reduce_default_tests.log
ECG_REDUCE_WIDE=2 ECG_REDUCE_WIDE_MIN=48 timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  tests/test_resnet_engine_gpu.py -k "grads" > gpurun_out/reduce_knob_tests2.log 2>&1 || { tail -30 gpurun_out/reduce_knob_tests2.log; exit 1; }
tail -1 gpurun_out/reduce_knob_tests2.log
bash scripts/ab_resnet_cfgs.sh 3 "base|X=0" "wide128|ECG_REDUCE_WIDE=2" "wide48|ECG_REDUCE_WIDE=2 ECG_REDUCE_WIDE_MIN=48" "wide20|ECG_REDUCE_WIDE=2 ECG_REDUCE_WIDE_MIN=20"
