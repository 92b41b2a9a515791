#!/bin/bash
# One GPU-box session: tests, smoke, bench, rocprof.  Every GPU step has its own time limit; a crash,
# abort or timeout (exit >= 124 or signal) stops the session, an ordinary test failure (exit 1) does not.
# Usage (from the repo root on the box): bash scripts/gpu_session.sh [steps...]
#   steps: tests smoke bench prof  (default: all)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
STEPS=${*:-"tests smoke bench prof"}

run() {  # run <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2; shift 2
  echo "=== [$name] $(date +%T) $*"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "!!! [$name] crashed/timed out (rc=$rc): stopping the session"
    exit $rc
  fi
  return 0
}

python csrc/build.py > "$OUT/build.log" 2>&1 || { cat "$OUT/build.log"; exit 2; }
for s in $STEPS; do
  case $s in
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 500 --warmup 100 ;;
    prof)
      export TMPDIR=/tmp
      run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
        python3 bench.py --steps 200 --warmup 50 --no-extras
      ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "=== session done $(date +%T)"
