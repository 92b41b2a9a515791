set -u
run() {  # run <label> <env...>
  local label=$1; shift
  timeout -k 10 300 env "$@" python bench.py --model resnet1d34 --steps 60 --warmup 10 --no-extras > gpurun_out/ab_$label.log 2>&1 || exit 1
  echo "$label $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$label.log)"
}
run nst2 ECG_CONV_NST=2
run nst3 ECG_CONV_NST=3
run nst3_cap16 ECG_CONV_NST=3 ECG_WGRAD_MAX_SPLITS=16
run nst3_cap8 ECG_CONV_NST=3 ECG_WGRAD_MAX_SPLITS=8
run nst2b ECG_CONV_NST=2
run nst3b ECG_CONV_NST=3
