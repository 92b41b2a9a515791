# rocprofv3 --kernel-trace --stats of the ResNet bench in the current tree and in _abtree/base (scripts/ab_tree.sh prep)
set -o pipefail
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
R=$PWD; mkdir -p $R/gpurun_out/r5_${PROF_TAG:-s6prof}
for t in cur base; do
  d=$R; [ $t = base ] && d=$R/_abtree/base
  (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r5_${PROF_TAG:-s6prof}/$t -o k -- python3 bench.py --model resnet1d34 --steps 10 --warmup 3 --no-extras > $R/gpurun_out/r5_${PROF_TAG:-s6prof}/$t.log 2>&1) || exit $?
done
