#!/bin/bash
# GPU measurement session on one MI355X (run by gpurun from the repo root):
#   bash scripts/gpu_session.sh <tag> <steps...>
# steps (any subset, in order): tests smoke bench bench20 resnet | probe bnprobe convtest enginetest |
#   module1 module1f module2 m2trace module3 | libab (LIBS=...) envab (ENVS=...) finab tapab | pmc tappmc tinypmc stats timeline timeline0
# Every GPU step runs under its own time limit; a crash, abort or timeout ends the session.
set -u
cd "$(dirname "$0")/.."
TAG=${1:-base}
shift
OUT=gpurun_out/${ECG_ROUND:-r6}_$TAG
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <timeout_s> <cmd...>
  local name=$1 tmo=$2
  shift 2
  echo "=== [$name] $(date +%T)"
  timeout -k 10 "$tmo" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 4 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "!!! [$name] rc=$rc: stopping"
    exit $rc
  fi
  if [ $rc -eq 1 ]; then echo "!!! [$name] failed (rc=1)"; fi
}
smi() { rocm-smi --showclocks --showpower --showtemp > "$OUT/smi_$1.txt" 2>&1 || true; }
{ hostname; rocm-smi --showserial --showproductname 2>/dev/null | grep -iE "serial|card series" | head -4; } > "$OUT/host.txt" 2>&1
smi start
for s in "$@"; do
  case $s in
    tests)
      step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      for i in 1 2 3; do step bench20_$i 300 python bench.py --steps 20 --warmup 5; done
      step bench500 300 python bench.py --steps 500 --warmup 100 --no-extras ;;
    bench20)
      for i in 1 2 3; do step bench20_$i 300 python bench.py --steps 20 --warmup 5 --no-extras; done ;;
    resnet)
      for i in 1 2 3; do step resnet_$i 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras; done ;;
    probe)
      step probe 300 python scripts/r4_conv_probe.py 30 1024,4096 ;;
    diag)
      step diag 300 python scripts/diag_step_phases.py ;;
    roundfix)  # ENVS="A=1 ...": fixed vs per-step cost of a round replay, default and each setting
      step roundfix0 120 python scripts/diag_round_fixed.py
      for e in ${ENVS:-}; do step "roundfix_${e}" 120 env $e python scripts/diag_round_fixed.py; done ;;
    m1trace)  # Module 1 B=128: A0 vs A3 compute ranges under a kernel + HIP API + marker trace
      export TMPDIR=/tmp
      step m1trace 400 rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d "$OUT/m1trace" \
        -o t -- python3 scripts/trace_module1_b128.py run
      step m1parse 120 python scripts/trace_module1_b128.py parse "$OUT/m1trace" ;;
    headm)
      step headm 120 python scripts/diag_head_m.py ;;
    bnprobe)
      step bnprobe 300 python scripts/r4_bn_probe.py 50 ;;
    convtest)
      step convtest 600 python -u -m pytest tests/test_conv_mc_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    tinytest)
      step tinytest 400 python -u -m pytest tests/test_fused_tiny_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ;;
    tailtest)
      step tailtest 300 python -u -m pytest tests/test_resnet_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "large_batch or depth34_well" ;;
    enginetest)
      step enginetest 900 python -u -m pytest tests/test_resnet_engine_gpu.py tests/test_resnet_trainer_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    module1)
      step shard_prep 300 python shard_prep.py --dataset synthetic
      step module1 1000 python bench_locality.py --batch-sizes 64 128 256 512 --reps 5 --results-dir "$OUT/modules" ;;
    module1f)  # A0-A5 with the fused HIP training step: the data path without the eager step's launches
      [ -d data/shards ] || step shard_prep 300 python shard_prep.py --dataset synthetic
      step module1f 1000 python bench_locality.py --compute fused --batch-sizes 64 128 256 512 --reps 9 --reps-large 15 \
        --results-dir "$OUT/modules" ;;
    module2)
      step module2 900 python benchmark_part_2.py --results-dir "$OUT/modules" ;;
    m2host)  # Module-2 single-call host settings A/B (GPU part only): spin-wait sync x timing-thread pin
      for r in 1 2; do for sp in 1 0; do for pin in late early; do
        ECG_M2_SPIN=$sp ECG_M2_PIN=$pin step m2host_s${sp}_${pin}_$r 300 python benchmark_part_2.py --no-cpu \
          --results-dir "$OUT/m2host_s${sp}_${pin}_$r"
      done; done; done ;;
    m2trace)  # which MIOpen kernels / HIP calls torch.nn.Conv1d runs per Module-2 cell
      export TMPDIR=/tmp
      step m2trace 400 rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d "$OUT/m2trace" \
        -o t -- python3 scripts/trace_module2_miopen.py run
      step m2parse 120 python scripts/trace_module2_miopen.py parse "$OUT/m2trace"
      rm -rf "$OUT/m2trace" ;;  # the raw HIP-API trace exceeds what gpurun copies back; the parse is the record
    module3)
      [ -d data/shards ] || step shard_prep 300 python shard_prep.py --dataset synthetic
      step pseudo_fl 600 python part3_mpi_gpu_train.py --steps 200 --results-csv "$OUT/modules/part3_mpi_cuda_results.csv"
      step fedavg 600 python part3_fedavg_overlap_mpi_gpu.py --data-root data/shards --rounds 5 --local-steps 50 \
        --config both --results-csv "$OUT/modules/fedavg_results_w1.csv"
      step plots 300 python plot_results.py --results-dir "$OUT/modules" ;;
    dist2)  # two ranks sharing the one GPU over gloo (RCCL needs one GPU per rank): the N>1 bench path on real
            # kernels - self-launch, per-rank placement, timing bracket, cross-rank weight self-check
      for ov in none tail; do
        step dist2_tiny_$ov 300 env ECG_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 100 --warmup 10 \
          --overlap $ov --no-extras
      done
      step dist2_resnet 300 env ECG_DIST_BACKEND=gloo python bench.py --gpus 2 --model resnet1d18 --steps 10 \
        --warmup 3 --batch-size 256 --no-extras ;;
    libab)  # LIBS="a b c": interleaved ResNet runs against _ablib/<a>, _ablib/<b>, ...
      for r in 1 2 3; do for v in ${LIBS}; do
        ECG_LIB_DIR=$PWD/_ablib/$v step resnet_lib${v}_$r 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
      done; done ;;
    tinylib)  # LIBS="a b": interleaved TinyECG K=20 / K=500 runs against _ablib/<a>, _ablib/<b>
      for r in 1 2 3 4; do for v in ${LIBS}; do
        ECG_LIB_DIR=$PWD/_ablib/$v step tiny20_lib${v}_$r 300 python bench.py --steps 20 --warmup 5 --no-extras
      done; done
      for v in ${LIBS}; do
        ECG_LIB_DIR=$PWD/_ablib/$v step tiny500_lib${v} 300 python bench.py --steps 500 --warmup 100 --no-extras
      done ;;
    tinyenv)  # ENVS="A=1 ...": interleaved TinyECG K=20 runs, default vs each setting
      for r in 1 2 3 4; do
        step tiny20_env0_$r 300 python bench.py --steps 20 --warmup 5 --no-extras
        for e in ${ENVS}; do step "tiny20_env_${e}_$r" 300 env $e python bench.py --steps 20 --warmup 5 --no-extras; done
      done ;;
    finab)  # fused BatchNorm finalize vs the separate one-launch finalize
      for r in 1 2 3; do
        ECG_BN_TAIL=1 step resnet_tail1_$r 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
        ECG_BN_TAIL=0 step resnet_fin1_$r 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
      done ;;
    envab)  # ENVS="A=1 B=2" pairs: interleaved runs, default vs each setting
      for r in 1 2 3; do
        step resnet_env0_$r 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
        for e in ${ENVS}; do env $e python -c pass && step "resnet_env_${e}_$r" 300 env $e python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras; done
      done ;;
    tappmc)
      export TMPDIR=/tmp
      step pmc_tap1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
        --kernel-trace --output-format csv -d "$OUT/pmc_tap1" -o p -- python3 scripts/r4_conv_probe.py 5 1024
      step pmc_tap2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv \
        -d "$OUT/pmc_tap2" -o p -- python3 scripts/r4_conv_probe.py 5 1024 ;;
    coldprobe)  # conv time with operands in HBM (a buffer ring larger than the Infinity Cache) vs cache-resident
      step coldprobe 300 python scripts/conv_cold_probe.py 24 ;;
    probe64)  # isolated conv timings with the persistent 64-channel tap kernel on / off
      for m in 1 0; do ECG_CONV_TAP64=$m step probe64_$m 300 python scripts/r4_conv_probe.py 30 1024; done ;;
    tapab)
      for m in 0 2; do ECG_CONV_TAP=$m step probe_tap$m 300 python scripts/r4_conv_probe.py 30 1024; done
      for r in 1 2; do for m in 0 1 2; do
        ECG_CONV_TAP=$m step resnet_tap${m}_$r 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
      done; done ;;
    pmc)
      export TMPDIR=/tmp
      step pmc_resnet 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 \
        SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
        -d "$OUT/pmc_resnet" -o p -- python3 bench.py --model resnet1d34 --steps 3 --warmup 2 --no-extras
      step pmc_resnet2 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
        SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv \
        -d "$OUT/pmc_resnet2" -o p -- python3 bench.py --model resnet1d34 --steps 3 --warmup 2 --no-extras ;;
    stats)
      export TMPDIR=/tmp
      step prof_tiny 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_tiny" -o tiny -- \
        python3 bench.py --steps 200 --warmup 50 --no-extras
      step prof_resnet 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_resnet" -o resnet -- \
        python3 bench.py --model resnet1d34 --steps 10 --warmup 3 --no-extras ;;
    timeline0)
      export TMPDIR=/tmp
      ECG_RESNET_SIDE=0 step timeline0 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline0" -o tl -- \
        python3 scripts/resnet_timeline.py run ;;
    timeline)
      export TMPDIR=/tmp
      step timeline 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/timeline" -o tl -- \
        python3 scripts/resnet_timeline.py run
      step prof_resnet 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_resnet" -o resnet -- \
        python3 bench.py --model resnet1d34 --steps 10 --warmup 3 --no-extras ;;
    queues)  # stream -> hardware-queue audit of the N>1 layout (compute, side lane, comm, RCCL) under a kernel trace
      export TMPDIR=/tmp
      step queues 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/queues" -o q -- \
        python3 scripts/probe_stream_queues.py run
      step queues_parse 120 python scripts/probe_stream_queues.py parse "$OUT/queues"
      ECG_RCCL_HIGH_PRIORITY=0 step queues_np 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/queues_np" \
        -o q -- python3 scripts/probe_stream_queues.py run
      step queues_np_parse 120 python scripts/probe_stream_queues.py parse "$OUT/queues_np" ;;
    tinypmc)
      export TMPDIR=/tmp
      step pmc_tiny 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES \
        SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --output-format csv -d "$OUT/pmc_tiny" -o p -- \
        python3 bench.py --steps 100 --warmup 20 --no-extras ;;
    *) echo "unknown step $s" ;;
  esac
done
smi end
echo "=== session $TAG done $(date +%T)"
