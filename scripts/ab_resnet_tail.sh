set -u
for i in 1 2; do
  timeout -k 10 300 python bench.py --model resnet1d34 --steps 60 --warmup 10 --no-extras > gpurun_out/ab_tail_$i.log 2>&1 || exit 1
  timeout -k 10 300 env ECG_BN_TAIL=0 python bench.py --model resnet1d34 --steps 60 --warmup 10 --no-extras > gpurun_out/ab_notail_$i.log 2>&1 || exit 1
done
grep -ho '"ms_per_step": [0-9.]*' gpurun_out/ab_*tail_*.log
