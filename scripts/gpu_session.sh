#!/bin/bash
# One GPU-box session: tests, smoke, bench, rocprof.  Every GPU step has its own time limit; a crash,
# abort or timeout (exit >= 124 or signal) stops the session, an ordinary test failure (exit 1) does not.
# Usage (from the repo root on the box): bash scripts/gpu_session.sh [steps...]
#   steps: tests smoke bench bench20 diag_g1 modules prof  (default: tests smoke bench prof)
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
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 500 --warmup 100 ;;
    bench20) run bench20 300 python bench.py --steps 20 --warmup 5
             run bench20b 300 python bench.py --steps 20 --warmup 5 --no-extras
             run bench500 300 python bench.py --steps 500 --warmup 100 --no-extras ;;
    resnet) run bench_resnet34 600 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras ;;
    resnet_tests) run resnet_tests 600 python -u -m pytest tests/test_resnet_engine_gpu.py tests/test_conv_mc_gpu.py \
                    -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    mt_ab) for r in a b; do
             for v in 0 1 2; do
               run bench_resnet34_mt${v}$r 300 env ECG_CONV_MT=$v python bench.py --model resnet1d34 --steps 20 \
                 --warmup 5 --no-extras
             done
           done
           run op_profile_mt1 300 env ECG_CONV_MT=1 python scripts/resnet_op_profile.py 34 1024
           run op_profile_mt2 300 env ECG_CONV_MT=2 python scripts/resnet_op_profile.py 34 1024 ;;
    diag_g1) run diag_g1 600 python scripts/diag_g1_overlap.py "$OUT/diag_g1" ;;
    diag_region) run diag_region 300 python scripts/diag_timed_region.py 20 9 ;;
    timeline)
      export TMPDIR=/tmp
      run resnet_tl 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tl" -o tl -- \
        python3 scripts/resnet_timeline.py run
      ;;
    bench_n2) run bench_n2_gloo 300 env ECG_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 \
                --no-extras ;;
    knob_ab)
      for r in a b; do
        for kv in "X=0" "ECG_CONV_BIG=0" "ECG_CONV_BIG=2" "ECG_CONV_V128=1" "ECG_CONV_V128=2" "ECG_CONV_NST=3" \
                  "ECG_WGRAD_MAX_SPLITS=48" "ECG_WGRAD_MAX_SPLITS=96" "ECG_CONV_MT=2" "ECG_CONV_NBUF=2"; do
          run "knob_${kv}_$r" 300 env $kv python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
        done
      done ;;
    hbm_bench)
      run bench_resnet34_64gb 600 python bench.py --model resnet1d34 --max-windows 32000000 --steps 60 --warmup 10 \
        --no-extras
      run bench_tiny_64gb 600 python bench.py --max-windows 32000000 --steps 500 --warmup 100 --no-extras ;;
    conv_stats) run conv_stats 300 python scripts/conv_stats_micro.py ;;
    k20_series)
      for i in 1 2 3 4; do run k20_$i 300 python bench.py --steps 20 --warmup 5 --no-extras; done
      sleep 5
      for i in 5 6; do run k20_$i 300 python bench.py --steps 20 --warmup 5 --no-extras; done ;;
    flag_tests) run flag_tests 300 python -u -m pytest tests/test_ops_gpu.py -k "flag_call" -x -v -p no:cacheprovider \
                  --timeout 120 --timeout-method thread ;;
    flag_ab) for c in 3 4 5 0 3 4 5; do run diag_call_cfg$c 300 env ECG_CONV1D_FLAG_CFG=$c python scripts/diag_conv1d_call.py; done ;;
    ops_tests) run ops_tests 300 python -u -m pytest tests/test_ops_gpu.py -x -v -p no:cacheprovider --timeout 120 \
                 --timeout-method thread ;;
    maskz_ab) for r in a b c; do for v in 0 1; do
                run maskz_${v}_$r 300 env ECG_DGRAD_MASK_FROM_Z=$v python bench.py --model resnet1d34 --steps 60 \
                  --warmup 10 --no-extras
              done; done ;;
    rpt_ab) for r in a b c; do for v in 0 4; do
              run rpt_${v}_$r 300 env ECG_BN_APPLY_RPT=$v python bench.py --model resnet1d34 --steps 60 --warmup 10 \
                --no-extras
            done; done ;;
    nst_ab) for r in a b; do for kv in "X=0" "ECG_CONV_V128=1" "ECG_CONV_NST=3" "ECG_CONV_V128=3"; do
              run "nst_${kv}_$r" 300 env $kv python bench.py --model resnet1d34 --steps 60 --warmup 10 --no-extras
            done; done
            for kv in "X=0" "ECG_CONV_V128=1" "ECG_CONV_NST=3"; do
              run "micro_${kv}" 120 env $kv python scripts/conv_stats_micro.py
            done ;;
    fold_ab) for r in a b c; do for v in 0 1 2; do
               run fold_${v}_$r 300 env ECG_BN_FOLD=$v python bench.py --model resnet1d34 --steps 60 --warmup 10 \
                 --no-extras
             done; done ;;
    split_ab) for r in a b c; do for v in 64 48 40; do
                run split_${v}_$r 300 env ECG_WGRAD_MAX_SPLITS=$v python bench.py --model resnet1d34 --steps 60 \
                  --warmup 10 --no-extras
              done; done ;;
    op_prof) run op_profile_mt0 300 env ECG_CONV_MT=0 python scripts/resnet_op_profile.py 34 1024
             run op_profile_mt1 300 env ECG_CONV_MT=1 python scripts/resnet_op_profile.py 34 1024 ;;
    mt_tests) run mt_tests 600 python -u -m pytest tests/test_conv_mc_gpu.py -k "stats_multi_tile" \
                tests/test_resnet_engine_gpu.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    diag_call) run diag_overhead 300 python scripts/diag_bench_overhead.py
               run diag_conv1d_call 300 python scripts/diag_conv1d_call.py ;;
    diag_resnet) run diag_resnet 600 python scripts/diag_resnet_numerics.py ;;
    tiny_tests) run tiny_tests 600 python -u -m pytest tests/test_fused_tiny_gpu.py -x -v -p no:cacheprovider \
                  --timeout 120 --timeout-method thread ;;
    diag_phases) run diag_phases 600 python scripts/diag_step_phases.py ;;
    diag_pf) run diag_pf 300 python scripts/diag_prefrag.py ;;
    diag_labl) run diag_labl 300 python scripts/diag_labl.py ;;
    bench_pref) run bench_pref1 300 python bench.py --steps 500 --warmup 100 --no-extras
                run bench_pref0 300 env ECG_TINY_PREFETCH=0 python bench.py --steps 500 --warmup 100 --no-extras
                run bench_pref1b 300 python bench.py --steps 500 --warmup 100 --no-extras
                run bench_pref0b 300 env ECG_TINY_PREFETCH=0 python bench.py --steps 500 --warmup 100 --no-extras ;;
    bench_wt) run bench_wt0 300 python bench.py --steps 500 --warmup 100 --no-extras
              run bench_wt1 300 env ECG_TINY_SLAB_WT=1 python bench.py --steps 500 --warmup 100 --no-extras
              run bench_wt0b 300 python bench.py --steps 500 --warmup 100 --no-extras
              run bench_wt1b 300 env ECG_TINY_SLAB_WT=1 python bench.py --steps 500 --warmup 100 --no-extras ;;
    bench_ab) run bench_pf 300 python bench.py --steps 500 --warmup 100 --no-extras
              run bench_lds 300 env ECG_TINY_PREFRAG=0 python bench.py --steps 500 --warmup 100 --no-extras
              run bench_pf20 300 python bench.py --steps 20 --warmup 5 --no-extras ;;
    bench_graph) for r in a b; do
                   run bench_g1_20$r 300 python bench.py --steps 20 --warmup 5 --no-extras
                   run bench_g0_20$r 300 env ECG_TINY_GRAPH=0 python bench.py --steps 20 --warmup 5 --no-extras
                   run bench_g1_500$r 300 python bench.py --steps 500 --warmup 100 --no-extras
                   run bench_g0_500$r 300 env ECG_TINY_GRAPH=0 python bench.py --steps 500 --warmup 100 --no-extras
                 done ;;
    hbm) run hbm 600 python -m crossscale_ecg.bench.hbm --gb 16 --dir /tmp/ecg_hbm_shards --cleanup ;;
    module2) mkdir -p gpurun_out/results
             run module2 600 python benchmark_part_2.py --results-dir gpurun_out/results --batch-scaling ;;
    modules)
      R=gpurun_out/results
      mkdir -p $R
      run module2 600 python benchmark_part_2.py --results-dir $R --batch-scaling
      run module1 900 python bench_locality.py --batch-sizes 64 128 256 512 --iters 100 --num-workers 4 \
        --shard-dir /tmp/ecg_shards --results-dir $R
      run module1_fused 600 python bench_locality.py --batch-sizes 256 --iters 100 --num-workers 4 --compute fused \
        --shard-dir /tmp/ecg_shards --results-dir $R/fused_compute
      run pseudo_fl 600 python part3_mpi_gpu_train.py --steps 200 --synthetic-windows 20000 \
        --results-csv $R/part3_mpi_cuda_results.csv --quiet
      run fedavg1 600 python part3_fedavg_overlap_mpi_gpu.py --synthetic-windows 20000 --rounds 5 \
        --local-steps 50 --config both --results-csv $R/fedavg_results_w1.csv
      run plots 300 python plot_results.py --results-dir $R
      ;;
    pmc)
      export TMPDIR=/tmp
      timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
      P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD"
      run pmc1 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$OUT/pmc1" -o tiny -- python3 scripts/pmc_tiny_step.py
      run pmc2 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d "$OUT/pmc2" -o tiny -- python3 scripts/pmc_tiny_step.py
      ;;
    conv_ab) run conv_picker 120 python scripts/conv_micro.py
             for t in 64x64 128x64 128x128 256x256; do run conv_$t 120 env ECG_CONV_TILE=$t python scripts/conv_micro.py; done ;;
    conv_v128) for v in 0 1 2 3; do run conv_v128_$v 120 env ECG_CONV_V128=$v python scripts/conv_micro.py; done ;;
    conv_pmc)
      export TMPDIR=/tmp
      P3="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY"
      run conv_pmc 120 rocprofv3 --pmc $P3 --kernel-trace --output-format csv -d "$OUT/conv_pmc" -o conv -- python3 scripts/conv_micro.py
      ;;
    prof)
      export TMPDIR=/tmp
      run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
        python3 bench.py --steps 200 --warmup 50 --no-extras
      ;;
    prof_resnet)
      export TMPDIR=/tmp
      run rocprof_resnet 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_resnet" -o resnet -- \
        python3 bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
      ;;
    wgrad_ab) run wgrad_ts0 120 env ECG_WGRAD_TS=0 python scripts/wgrad_micro.py
              for kv in "ECG_WGRAD_TS_NST=4 ECG_WGRAD_TS_WGS=256" "ECG_WGRAD_TS_NST=4 ECG_WGRAD_TS_WGS=512" \
                        "ECG_WGRAD_TS_NST=3 ECG_WGRAD_TS_WGS=512" "ECG_WGRAD_TS_NST=2 ECG_WGRAD_TS_WGS=512" \
                        "ECG_WGRAD_TS_NST=4 ECG_WGRAD_TS_WGS=1024"; do
                run "wgrad_${kv// /_}" 120 env $kv python scripts/wgrad_micro.py
              done ;;
    conv_tests) run conv_tests 600 python -u -m pytest tests/test_conv_mc_gpu.py -x -v -p no:cacheprovider --timeout 300 \
                  --timeout-method thread ;;
    resnet_ab) for r in a b; do
                 run resnet_ts1_$r 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
                 run resnet_ts0_$r 300 env ECG_WGRAD_TS=0 ECG_REDUCE_WIDE=0 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
               done ;;
    conv3_ab) for v in 0 1 3; do run conv3_v128_$v 120 env ECG_CONV_V128=$v python scripts/conv_micro.py; done
              run conv3_nst3 120 env ECG_CONV_NST=3 python scripts/conv_micro.py
              for kv in "X=0" "ECG_CONV_V128=1" "ECG_CONV_NST=3" "ECG_CONV_V128=1 ECG_CONV_NST=3"; do
                run "r34_${kv// /_}" 300 env $kv python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
              done ;;
    wr_ab) run conv_wr1 120 python scripts/conv_micro.py
           run conv_wr0 120 env ECG_CONV_WR=0 python scripts/conv_micro.py
           for r in a b; do
             run r34_wr1_$r 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
             run r34_wr0_$r 300 env ECG_CONV_WR=0 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
           done ;;
    r34_matrix) for r in a b; do
                  for kv in "ECG_CONV_WR=0 ECG_WGRAD_TS=0 ECG_REDUCE_WIDE=0" "ECG_CONV_WR=0 ECG_WGRAD_TS=0" \
                            "ECG_CONV_WR=0 ECG_REDUCE_WIDE=0" "ECG_CONV_WR=0" "ECG_CONV_WR=64" \
                            "ECG_CONV_WR=64 ECG_WGRAD_TS=0 ECG_REDUCE_WIDE=0"; do
                    run "m_${kv// /_}_$r" 300 env $kv python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
                  done
                done ;;
    head_ab) for r in a b c; do for h in 0 1 2 4; do
               run "head${h}_$r" 300 env ECG_TINY_HEAD=$h python bench.py --steps 20 --warmup 5 --no-extras
             done; done
             for h in 0 2; do run "head${h}_500" 300 env ECG_TINY_HEAD=$h python bench.py --steps 500 --warmup 100 --no-extras; done ;;
    gather_ab) for r in a b c; do for g in 0 1; do
                 run "gather${g}_$r" 300 env ECG_TINY_GATHER=$g python bench.py --steps 20 --warmup 5 --no-extras
               done; done
               for g in 0 1; do run "gather${g}_500" 300 env ECG_TINY_GATHER=$g python bench.py --steps 500 --warmup 100 --no-extras; done ;;
    tiny_tests) run tiny_tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_tiny_gpu.py ;;
    m1reps) R=gpurun_out/r3mod; mkdir -p $R
            run module1_r5 1100 python bench_locality.py --batch-sizes 64 128 256 512 --iters 100 --num-workers 4 \
              --shard-dir /tmp/ecg_shards --results-dir $R --reps 5 ;;
    m1pin) R=gpurun_out/r3mod_pin; mkdir -p $R
           run module1_pin_r5 1100 python bench_locality.py --batch-sizes 64 128 256 512 --iters 100 --num-workers 4 \
             --shard-dir /tmp/ecg_shards --results-dir $R --reps 5 --pin-thread ;;
    m23) R=gpurun_out/r3mod; mkdir -p $R
         run module2 600 python benchmark_part_2.py --results-dir $R --batch-scaling
         run pseudo_fl 600 python part3_mpi_gpu_train.py --steps 200 --synthetic-windows 20000 \
           --results-csv $R/part3_mpi_cuda_results.csv --quiet
         run fedavg1 600 python part3_fedavg_overlap_mpi_gpu.py --synthetic-windows 20000 --rounds 5 \
           --local-steps 50 --config both --results-csv $R/fedavg_results_w1.csv ;;
    prof_gather) export TMPDIR=/tmp
      for g in 0 1; do
        export ECG_TINY_GATHER=$g
        run prof_gather$g 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_gather$g" -o run -- \
          python3 bench.py --steps 500 --warmup 100 --no-extras
      done
      unset ECG_TINY_GATHER ;;
    prof_resnet) export TMPDIR=/tmp
      run prof_resnet 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_resnet" -o run -- \
        python3 bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras ;;
    kscan) run kscan_l3 300 python scripts/conv_kscan.py 1024 32 256
           run kscan_l4 300 python scripts/conv_kscan.py 1024 16 512
           run kscan_l2 300 python scripts/conv_kscan.py 1024 63 128
           run kscan_l3_v1 300 env ECG_CONV_V128=1 python scripts/conv_kscan.py 1024 32 256
           run kscan_l3_v2 300 env ECG_CONV_V128=2 python scripts/conv_kscan.py 1024 32 256 ;;
    epi_ab) run resnet_tests_epi 600 python -u -m pytest tests/test_resnet_engine_gpu.py tests/test_conv_mc_gpu.py \
              -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
            for r in a b c; do
              run "resnet_epi_$r" 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
            done
            run op_profile 300 python scripts/resnet_op_profile.py 34 1024
            export TMPDIR=/tmp
            run prof_resnet_tl 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_resnet3" -o run -- \
              python3 bench.py --model resnet1d34 --steps 10 --warmup 3 --no-extras
            export ECG_BN_TAIL=0
            run prof_resnet_tail0 400 rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof_resnet3_tail0" -o run -- \
              python3 bench.py --model resnet1d34 --steps 10 --warmup 3 --no-extras
            unset ECG_BN_TAIL ;;
    train_diag) for kv in "X=0" "ECG_WGRAD_TS=0" "ECG_REDUCE_WIDE=0" "ECG_RESNET_SIDE=0" "ECG_BN_TAIL=0" "ECG_CONV_DMA=0" \
                         "ECG_CONV_MT=0"; do
                  run "train_${kv}" 120 env $kv python scripts/diag_train_progress.py 18 64
                done ;;
    resnet_tests_all) run resnet_tests_all 900 python -u -m pytest tests/test_resnet_engine_gpu.py tests/test_conv_mc_gpu.py \
                        tests/test_resnet_trainer_gpu.py -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    tail_ab) for r in a b; do for g in 0 8 16 32; do
               run "tailgs${g}_$r" 300 env ECG_BN_TAIL_GS=$g python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
             done; done ;;
    epi_tail_ab) for r in a b c; do
                   run "base_$r" 300 env ECG_LIB_DIR=$PWD/_ablib/base ECG_BN_TAIL_GS=-1 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
                   run "new_$r" 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
                   run "new_gsold_$r" 300 env ECG_BN_TAIL_GS=-1 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
                 done ;;
    tiny_ab) for r in a b c; do
               run "tbase500_$r" 300 env ECG_LIB_DIR=$PWD/_ablib/base python bench.py --steps 500 --warmup 100 --no-extras
               run "tnew500_$r" 300 python bench.py --steps 500 --warmup 100 --no-extras
               run "tbase20_$r" 300 env ECG_LIB_DIR=$PWD/_ablib/base python bench.py --steps 20 --warmup 5 --no-extras
               run "tnew20_$r" 300 python bench.py --steps 20 --warmup 5 --no-extras
             done ;;
    tiny_pmc) export TMPDIR=/tmp
      P2="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD"
      run pmc2_new 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d "$OUT/pmc2_new" -o tiny -- python3 scripts/pmc_tiny_step.py
      export ECG_LIB_DIR=$PWD/_ablib/base
      run pmc2_base 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d "$OUT/pmc2_base" -o tiny -- python3 scripts/pmc_tiny_step.py
      unset ECG_LIB_DIR ;;
    tail2_ab) for r in a b c; do
                run "t2base_$r" 300 env ECG_LIB_DIR=$PWD/_ablib/base python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
                run "t2new_$r" 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
                run "t2gs4_$r" 300 env ECG_BN_TAIL_GS=4 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
              done ;;
    wc_test) run wc_test 300 python -u -m pytest tests/test_resnet_engine_gpu.py -k "well_conditioned or training_progress or bn_tail" -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    epi2_ab) for r in a b c d; do
               run "e2base_$r" 300 env ECG_LIB_DIR=$PWD/_ablib/base python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
               run "e2new_$r" 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
             done ;;
    dil_ab) for r in a b c d; do
              run "dil0_$r" 300 env ECG_CONV_DMA_DIL=0 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
              run "dil1_$r" 300 python bench.py --model resnet1d34 --steps 20 --warmup 5 --no-extras
            done ;;
    m23p) R=gpurun_out/r3mod; mkdir -p $R
          run module2 600 python benchmark_part_2.py --results-dir $R --batch-scaling
          run pseudo_fl 600 python part3_mpi_gpu_train.py --steps 200 --synthetic-windows 20000 \
            --results-csv $R/part3_mpi_cuda_results.csv --quiet
          run fedavg1 600 python part3_fedavg_overlap_mpi_gpu.py --synthetic-windows 20000 --rounds 5 \
            --local-steps 50 --config both --results-csv $R/fedavg_results_w1.csv
          run plots 300 python plot_results.py --results-dir $R ;;
    lib_ab) LIBB=${LIBB:-nnan}; for r in a b c d; do
              run "lb_cur500_$r" 300 python bench.py --steps 500 --warmup 100 --no-extras
              run "lb_${LIBB}500_$r" 300 env ECG_LIB_DIR=$PWD/_ablib/$LIBB python bench.py --steps 500 --warmup 100 --no-extras
              run "lb_cur20_$r" 300 python bench.py --steps 20 --warmup 5 --no-extras
              run "lb_${LIBB}20_$r" 300 env ECG_LIB_DIR=$PWD/_ablib/$LIBB python bench.py --steps 20 --warmup 5 --no-extras
            done ;;
    tiny_bench3) for r in a b c; do
                   run "tb500_$r" 300 python bench.py --steps 500 --warmup 100 --no-extras
                   run "tb20_$r" 300 python bench.py --steps 20 --warmup 5 --no-extras
                 done ;;
    tiny_pmc_valu) export TMPDIR=/tmp
      P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
      run pmcv_new 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d "$OUT/pmcv_new" -o tiny -- python3 scripts/pmc_tiny_step.py ;;
    env_ab) for r in a b c d; do
              run "ea_on500_$r" 300 python bench.py --steps 500 --warmup 100 --no-extras
              run "ea_off500_$r" 300 env $ENVA python bench.py --steps 500 --warmup 100 --no-extras
              run "ea_on20_$r" 300 python bench.py --steps 20 --warmup 5 --no-extras
              run "ea_off20_$r" 300 env $ENVA python bench.py --steps 20 --warmup 5 --no-extras
            done ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "=== session done $(date +%T)"
