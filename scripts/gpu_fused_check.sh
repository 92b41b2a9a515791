#!/bin/bash
# Short GPU check of the fused TinyECG step: its numerics tests, the phase diagnostic and the headline bench.
# Every GPU step has its own time limit; a crash/abort/timeout stops the script.
# Usage (repo root, on the GPU box): bash scripts/gpu_fused_check.sh [tag]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-check}
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_fused_tiny_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/t_fused_$TAG.log" 2>&1
rc=$?
tail -5 "$OUT/t_fused_$TAG.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/diag_step_phases.py > "$OUT/diag_$TAG.log" 2>&1 || exit $?
cat "$OUT/diag_$TAG.log"
timeout -k 10 300 python bench.py --steps 500 --warmup 100 --no-extras > "$OUT/bench_$TAG.log" 2>&1 || exit $?
cat "$OUT/bench_$TAG.log"
