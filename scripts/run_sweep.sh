#!/bin/bash
# FedAvg scaling sweep on ONE 8x MI355X node (reference TRUE_FL_M3/run_part3_sweep.sh: srun over 1/2/4/8
# nodes, 1 GPU each).  Here: torchrun, one process per GPU, RCCL over xGMI.
#   bash scripts/run_sweep.sh [DATA_ROOT]      (no DATA_ROOT: on-device synthetic windows)
# Env: WORLD_SIZES (default "1 2 4 8"), REPEATS (5), RESULTS_DIR (results), ECG_DIST_BACKEND=gloo to rehearse
# the sweep with several ranks sharing fewer GPUs (plumbing only: the timings are not a scaling measurement).
set -euo pipefail
cd "$(dirname "$0")/.."
export HSA_ENABLE_IPC_MODE_LEGACY=0
WORLD_SIZES=(${WORLD_SIZES:-1 2 4 8})
REPEATS=${REPEATS:-5}
DATA=${1:-}
RES=${RESULTS_DIR:-results}
mkdir -p "$RES"
for W in "${WORLD_SIZES[@]}"; do
  for R in $(seq 1 "$REPEATS"); do
    echo "=== world=$W repeat=$R"
    ARGS=(--batch-size 256 --rounds 5 --local-steps 50 --config both --max-windows 20000
          --results-csv "$RES/fedavg_results_w${W}.csv" --quiet)
    if [ -n "$DATA" ]; then ARGS+=(--data-root "$DATA"); else ARGS+=(--synthetic-windows 20000); fi
    timeout -k 10 900 python -m torch.distributed.run --nnodes 1 --nproc-per-node "$W" \
      --master-addr 127.0.0.1 --master-port $((29600 + W)) part3_fedavg_overlap_mpi_gpu.py "${ARGS[@]}"
  done
done
python plot_results.py --results-dir "$RES"
