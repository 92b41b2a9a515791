#!/bin/bash
# Per-layer conv microbench (LDS-DMA loop on and off) and one PMC pass per shape on the forward kernel.
# Usage (repo root, on the GPU box): bash scripts/gpu_conv_prof.sh [tag] [shapes]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-prof}
SHAPES=${2:-"l1 l3 l4"}
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv_mc_gpu.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/t_conv_$TAG.log" 2>&1 || { tail -30 "$OUT/t_conv_$TAG.log"; exit 1; }
tail -2 "$OUT/t_conv_$TAG.log"
for big in ${BIGS:-0 1 2}; do
  ECG_CONV_BIG=$big timeout -k 10 200 python scripts/conv_microbench.py > "$OUT/cmb_${TAG}_big$big.log" 2>&1 || exit $?
  echo "big=$big"; grep shape "$OUT/cmb_${TAG}_big$big.log"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
CNT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
for s in $SHAPES; do
  timeout -s KILL 90 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/pmc_${TAG}_$s" -o p -- python3 scripts/conv_one.py "$s" \
    > "$OUT/pmc_${TAG}_$s.log" 2>&1 || exit $?
done
echo done
