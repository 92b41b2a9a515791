#!/bin/bash
# End-of-round validation on one MI355X: GPU test suite, smoke, the driver's bench command (x3), K=500, ResNet1D-34,
# rocprofv3 kernel statistics of both benches.  Every GPU step under its own time limit; a crash/timeout ends it.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/final_r3
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== [$name] $(date +%T)"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!!! [$name] rc=$rc: stopping"; exit $rc; fi
}
python csrc/build.py > "$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 2; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2 3; do step bench20_$i 300 python bench.py --steps 20 --warmup 5; done
step bench500 300 python bench.py --steps 500 --warmup 100 --no-extras
for i in 1 2; do step resnet_$i 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras; done
export TMPDIR=/tmp
step prof_tiny 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tiny" -o tiny -- \
  python3 bench.py --steps 200 --warmup 50 --no-extras
step prof_resnet 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_resnet" -o resnet -- \
  python3 bench.py --model resnet1d34 --steps 10 --warmup 3 --no-extras
echo "=== final validation done $(date +%T)"
