# A/B of ResNet1D-34 B=1024 bench.py runs under environment settings: ab_resnet_env.sh NAME=ENV[,ENV...] ...
# (an empty ENV list = defaults); two interleaved repeats each, ms_per_step collected in gpurun_out/ab_env.txt
set -u
: > gpurun_out/ab_env.txt
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    timeout -k 10 300 env ${envs//,/ } python bench.py --model resnet1d34 --steps 60 --warmup 10 --no-extras \
      > gpurun_out/ab_env_${name}_$rep.log 2>&1 || exit 1
    echo "$name rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_env_${name}_$rep.log)" >> gpurun_out/ab_env.txt
  done
done
cat gpurun_out/ab_env.txt
