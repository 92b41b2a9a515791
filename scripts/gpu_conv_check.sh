#!/bin/bash
# GPU check of the MFMA conv kernels and the ResNet1D engine: numerics tests, then engine throughput with the
# LDS-DMA forward loop on and off (ECG_CONV_DMA).  Every GPU step has its own time limit.
# Usage (repo root, on the GPU box): bash scripts/gpu_conv_check.sh [tag]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-check}
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_conv_mc_gpu.py tests/test_resnet_engine_gpu.py -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/t_conv_$TAG.log" 2>&1
rc=$?
tail -5 "$OUT/t_conv_$TAG.log"
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
for dma in 1 0; do
  ECG_CONV_DMA=$dma timeout -k 10 300 python scripts/bench_resnet.py --backends engine --batches 1024,4096 \
    > "$OUT/resnet_${TAG}_dma$dma.log" 2>&1 || exit $?
  echo "dma=$dma"; grep model "$OUT/resnet_${TAG}_dma$dma.log"
done
