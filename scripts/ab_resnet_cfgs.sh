#!/bin/bash
# ResNet1D-34 B=1024 A/B over library builds and knobs, interleaved reps (one GPU call).
#   bash scripts/ab_resnet_cfgs.sh <reps> "<label>|<env assignments or X=0>" ...
# A label starting with "lib:<dir>" runs with ECG_LIB_DIR=_ablib/<dir>.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
reps=$1; shift
for r in $(seq 1 "$reps"); do
  for cfg in "$@"; do
    label=${cfg%%|*}; kv=${cfg#*|}
    extra=""
    case $label in lib:*) extra="ECG_LIB_DIR=$PWD/_ablib/${label#lib:}";; esac
    timeout -k 10 300 env $extra $kv python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras \
      > "gpurun_out/ab_${label//[:\/]/_}_$r.log" 2>&1
    rc=$?
    echo "[$label rep $r] rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_${label//[:\/]/_}_$r.log")"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
