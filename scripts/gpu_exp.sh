# The one GPU command file: every gpurun experiment is a preset of this script.
#   gpurun -- bash scripts/gpu_exp.sh <kind> [args...]
# Each GPU step has its own time limit and steps are chained with &&, so the first
# failure (fault, abort, timeout) ends the call. Logs land in gpurun_out/.
# kinds:
#   tests   [test paths]              GPU test tier (default: all of tests/) -> exp_tests.log
#   smoke                             __graft_entry__.smoke()           -> exp_smoke.log
#   check                             tests + smoke + short bench + rocprof kernel stats
#   bench   [bench.py args]           headline bench, JSON line         -> exp_bench.log
#   prof    [bench.py args]           rocprofv3 kernel stats of bench.py -> exp_prof/
#   pmc     "<counters>" [gbench args]  one PMC pass on gbench_forest.py -> exp_pmc/
#   roofline [gbench args]            kernel trace + the four PMC passes of the roofline table
#   phase                             per-phase k_nodes cycles (needs lib/libdml_hip_phase.so)
#   sweep   [sweep_tiers.py args]     forest tier sweep
#   configs [bench_configs.py args]   BASELINE configs 1/2/4/5
#   gbench  [gbench_forest.py args]   forest builder micro-bench
#   e2e                               bench.py --e2e local and over a world-1 process group
#   rccl                              world-1 RCCL tests + bench over the process group + rocprof
#   rehearse                          bench.py --gpus 2/4 sharing the one GPU over gloo
#   scaling                           scaling_sim.py at 2/4/8 ranks
#   gbrt                              BASELINE-style GBRT grid (bench_configs.py config 6) + its kernel trace
#   cluster                           world-1 RCCL runner test + config 5 and bench --e2e through the cluster runner
#   rccljob                           kernel trace of the world-1 RCCL cluster-runner test (RCCL kernels of real jobs)
#   svm     [svm_bench.py args]       SVC 50k x 20, 8 candidates x cv5 (+ its kernel stats)
#   envsweep "<settings>" <target>    one run of <target> per setting; a setting is a comma-separated
#                                     list of VAR=value (env) or LIB=<suffix> (lib/libdml_hip_<suffix>.so;
#                                     "cur" = the built library), settings separated by spaces, e.g.
#                                       envsweep "DML_LR_V4=1 DML_LR_V4=0" lrk
#                                       envsweep "LIB=cur LIB=cg2" lrk
#                                     targets: bench (bench.py --steps 10 --warmup 3), c6 (config 6),
#                                     lrk (lr_kernel_bench 10M x 1000 x 2560), lrbench (bench.py --config lr),
#                                     tiers (sweep_tiers.py forest build), c6prof (config 6 + top kernels),
#                                     c6rep (config 6, five back-to-back jobs in one process: seconds each)
#   whole                             kernel trace over the driver's exact bench command -> GPU busy
#   lrpmc                             the LR objective's PMC passes (MFMA busy, LDS, TCC, TA)
#   baseline                          round-start numbers: bench kernel stats, LR config 4, GBRT config 6, SVC
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
PYT="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
GB="scripts/gbench_forest.py"
kind=$1; shift
case "$kind" in
  tests)   timeout -k 10 900 $PYT -m gpu ${@:-tests} > gpurun_out/exp_tests.log 2>&1; rc=$?; tail -3 gpurun_out/exp_tests.log; exit $rc ;;
  smoke)   timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/exp_smoke.log 2>&1 && tail -1 gpurun_out/exp_smoke.log ;;
  check)   timeout -k 10 900 $PYT tests -m gpu > gpurun_out/exp_tests.log 2>&1 && tail -1 gpurun_out/exp_tests.log && \
           timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/exp_smoke.log 2>&1 && tail -1 gpurun_out/exp_smoke.log && \
           timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/exp_bench.log 2>&1 && tail -1 gpurun_out/exp_bench.log && \
           timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp_prof -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/exp_prof.log 2>&1 && echo PROF_OK ;;
  bench)   timeout -k 10 900 python -u bench.py "$@" > gpurun_out/exp_bench.log 2>&1 && tail -1 gpurun_out/exp_bench.log ;;
  prof)    timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp_prof -o run -- python3 bench.py "$@" > gpurun_out/exp_prof.log 2>&1 && echo PROF_OK ;;
  pmc)     ctrs=$1; shift; args=${*:-1000000 100 100 5}
           timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/exp_pmc -o p -- python3 $GB $args > gpurun_out/exp_pmc.log 2>&1 && echo PMC_OK ;;
  roofline) args=${*:-1000000 100 100 5}
           timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rf_kt -o p -- python3 $GB $args > gpurun_out/rf_kt.log 2>&1 && echo KT_OK && \
           timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/rf_a -o p -- python3 $GB $args > gpurun_out/rf_a.log 2>&1 && echo PA_OK && \
           timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/rf_b -o p -- python3 $GB $args > gpurun_out/rf_b.log 2>&1 && echo PB_OK && \
           timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/rf_c -o p -- python3 $GB $args > gpurun_out/rf_c.log 2>&1 && echo PC_OK && \
           timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/rf_d -o p -- python3 $GB $args > gpurun_out/rf_d.log 2>&1 && echo PD_OK ;;
  phase)   DML_HIP_LIB=cs230_distributed_machine_learning_amd/lib/libdml_hip_phase.so timeout -k 10 300 python -u scripts/phase_prof.py > gpurun_out/exp_phase.log 2>&1 && tail -3 gpurun_out/exp_phase.log ;;
  sweep)   timeout -k 10 900 python -u scripts/sweep_tiers.py "$@" > gpurun_out/exp_sweep.log 2>&1 && cat gpurun_out/exp_sweep.log ;;
  configs) timeout -k 10 900 python -u scripts/bench_configs.py "$@" > gpurun_out/exp_configs.log 2>&1 && cat gpurun_out/exp_configs.log ;;
  gbench)  timeout -k 10 600 python -u $GB "$@" > gpurun_out/exp_gbench.log 2>&1 && cat gpurun_out/exp_gbench.log ;;
  e2e)     timeout -k 10 900 python -u bench.py --e2e > gpurun_out/exp_e2e_local.log 2>&1 && tail -1 gpurun_out/exp_e2e_local.log && \
           DML_FORCE_PG=1 MASTER_PORT=29601 timeout -k 10 900 python -u bench.py --e2e > gpurun_out/exp_e2e_dist.log 2>&1 && tail -1 gpurun_out/exp_e2e_dist.log ;;
  rccl)    timeout -k 10 300 $PYT tests/test_rccl_gpu.py > gpurun_out/exp_rccl_test.log 2>&1 && tail -1 gpurun_out/exp_rccl_test.log && \
           DML_FORCE_PG=1 MASTER_PORT=29581 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/exp_rccl_bench.log 2>&1 && tail -1 gpurun_out/exp_rccl_bench.log | cut -c1-160 && \
           DML_FORCE_PG=1 MASTER_PORT=29582 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp_rccl_prof -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/exp_rccl_prof.log 2>&1 && echo PROF_OK ;;
  rehearse) export DML_SHARE_DEVICE=1 DML_DIST_BACKEND=gloo DML_HBM_BUDGET_GB=40
           timeout -k 10 400 python bench.py --gpus 2 --rows 250000 --steps 2 --warmup 1 --master-port 29611 > gpurun_out/exp_rh2.log 2>&1 && tail -1 gpurun_out/exp_rh2.log | cut -c1-330 && \
           timeout -k 10 400 python bench.py --gpus 4 --rows 250000 --steps 1 --warmup 1 --master-port 29612 > gpurun_out/exp_rh4.log 2>&1 && tail -1 gpurun_out/exp_rh4.log | cut -c1-330 ;;
  scaling) timeout -k 10 600 python -u scripts/scaling_sim.py --world 2,4,8 --steps 2 > gpurun_out/exp_scaling.log 2>&1 && cat gpurun_out/exp_scaling.log ;;
  gbrt)    timeout -k 10 600 python -u scripts/bench_configs.py --configs 6 > gpurun_out/exp_gbrt.log 2>&1 && tail -1 gpurun_out/exp_gbrt.log | cut -c1-300 && \
           timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp_gbrt_prof -o run -- python3 scripts/bench_configs.py --configs 6 > gpurun_out/exp_gbrt_prof.log 2>&1 && \
           python scripts/timeline.py gpurun_out/exp_gbrt_prof k_count_active > gpurun_out/exp_gbrt_busy.txt && rm -f gpurun_out/exp_gbrt_prof/*kernel_trace.csv && head -3 gpurun_out/exp_gbrt_busy.txt ;;
  cluster) timeout -k 10 300 $PYT tests/test_rccl_gpu.py > gpurun_out/exp_rccl_test.log 2>&1 && tail -1 gpurun_out/exp_rccl_test.log && \
           DML_FORCE_PG=1 MASTER_PORT=29602 timeout -k 10 600 python -u scripts/bench_configs.py --configs 5 > gpurun_out/exp_cfg5_dist.log 2>&1 && tail -1 gpurun_out/exp_cfg5_dist.log | cut -c1-300 && \
           DML_FORCE_PG=1 MASTER_PORT=29601 timeout -k 10 900 python -u bench.py --e2e > gpurun_out/exp_e2e_dist.log 2>&1 && tail -1 gpurun_out/exp_e2e_dist.log | cut -c1-300 ;;
  rccljob) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp_rccljob -o run -- python3 -m pytest -x -q tests/test_rccl_gpu.py > gpurun_out/exp_rccljob.log 2>&1 && \
           rm -f gpurun_out/exp_rccljob/*kernel_trace.csv && grep -i -c "nccl\|rccl" gpurun_out/exp_rccljob/run_kernel_stats.csv ;;
  lrprof)  args=${*:-10000000 1000 2560}
           timeout -k 10 300 python -u scripts/lr_kernel_bench.py $args > gpurun_out/exp_lrk.log 2>&1 && tail -1 gpurun_out/exp_lrk.log && \
           timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lr_kt -o p -- python3 scripts/lr_kernel_bench.py $args > gpurun_out/lr_kt.log 2>&1 && echo KT_OK && \
           timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lr_a -o p -- python3 scripts/lr_kernel_bench.py $args > gpurun_out/lr_a.log 2>&1 && echo PA_OK && \
           timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lr_b -o p -- python3 scripts/lr_kernel_bench.py $args > gpurun_out/lr_b.log 2>&1 && echo PB_OK && \
           timeout -k 10 400 python -u bench.py --config lr --steps 2 --warmup 1 > gpurun_out/exp_lrbench.log 2>&1 && tail -1 gpurun_out/exp_lrbench.log | cut -c1-1500 ;;
  svm)     timeout -k 10 300 python -u scripts/svm_bench.py "$@" > gpurun_out/exp_svm.log 2>&1 && tail -1 gpurun_out/exp_svm.log | cut -c1-400 && \
           timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp_svm_prof -o run -- python3 scripts/svm_bench.py "$@" > gpurun_out/exp_svm_prof.log 2>&1 && \
           rm -f gpurun_out/exp_svm_prof/*kernel_trace.csv && echo PROF_OK ;;
  baseline) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp_prof -o run -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/exp_prof.log 2>&1 && \
           rm -f gpurun_out/exp_prof/*kernel_trace.csv && echo PROF_OK && \
           timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > gpurun_out/exp_lr.log 2>&1 && tail -1 gpurun_out/exp_lr.log | cut -c1-200 && \
           timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/exp_c6.log 2>&1 && grep -o '"cv_fits_per_s[^,]*' gpurun_out/exp_c6.log && \
           timeout -k 10 300 python -u scripts/svm_bench.py > gpurun_out/exp_svm.log 2>&1 && tail -1 gpurun_out/exp_svm.log | cut -c1-400 ;;
  envsweep) settings=$1; target=$2; i=0
           for st in $settings; do
             i=$((i+1)); envs=(); lib=""
             for kv in ${st//,/ }; do
               case $kv in LIB=cur) lib="";; LIB=*) lib=cs230_distributed_machine_learning_amd/lib/libdml_hip_${kv#LIB=}.so;; *) envs+=("$kv");; esac
             done
             [ -n "$lib" ] && envs+=("DML_HIP_LIB=$lib")
             log=gpurun_out/sweep_${i}.log
             case $target in
               bench)   env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $log 2>&1 || exit 1
                        echo "[$st] $(grep -o '"value": [0-9.]*' $log | head -1)" ;;
               c6)      env "${envs[@]}" timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > $log 2>&1 || exit 1
                        echo "[$st] $(grep -o '"cv_fits_per_s[^,]*' $log)" ;;
               lrk)     env "${envs[@]}" timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > $log 2>&1 || exit 1
                        echo "[$st] $(tail -1 $log)" ;;
               lrbench) env "${envs[@]}" timeout -k 10 400 python -u bench.py --config lr --steps 3 --warmup 1 > $log 2>&1 || exit 1
                        echo "[$st] $(tail -1 $log | cut -c1-200)" ;;
               tiers)   env "${envs[@]}" timeout -k 10 300 python -u scripts/sweep_tiers.py > $log 2>&1 || exit 1
                        echo "[$st] $(grep build $log | tail -1 | cut -c1-80)" ;;
               c6rep)   env "${envs[@]}" DML_C6_REPEAT=5 timeout -k 10 400 python -u scripts/bench_configs.py --configs 6 > $log 2>&1 || exit 1
                        echo "[$st] $(grep -o 'repeat [0-9]: [0-9.]* s' $log | tr '\n' ' ') $(grep -o '"seconds": [0-9.]*' $log)" ;;
               c6prof)  env "${envs[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweep_prof$i -o run -- python3 scripts/bench_configs.py --configs 6 > $log 2>&1 || exit 1
                        rm -f gpurun_out/sweep_prof$i/*kernel_trace.csv
                        echo "[$st] $(grep -o '"cv_fits_per_s[^,]*' $log)"
                        python3 scripts/summarize_prof.py gpurun_out/sweep_prof$i > gpurun_out/sweep_prof$i.txt; sed -n 2,5p gpurun_out/sweep_prof$i.txt ;;
               *) echo "unknown sweep target $target"; exit 2 ;;
             esac
           done ;;
  whole)   s=$(date +%s.%N)
           timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wholebench -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/wb_bench.log 2>&1 || exit 1
           e=$(date +%s.%N)
           tail -1 gpurun_out/wb_bench.log | cut -c1-200
           python3 scripts/whole_run_busy.py gpurun_out/wholebench $(python3 -c "print($e-$s)") 5
           rm -rf gpurun_out/wholebench ;;
  lrpmc)   A=10000000
           timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lrpmc_a -o p -- python3 scripts/lr_kernel_bench.py $A 1000 2560 > gpurun_out/lrpmc_a.log 2>&1 && echo PA_OK && \
           timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lrpmc_b -o p -- python3 scripts/lr_kernel_bench.py $A 1000 2560 > gpurun_out/lrpmc_b.log 2>&1 && echo PB_OK && \
           timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/lrpmc_c -o p -- python3 scripts/lr_kernel_bench.py $A 1000 2560 > gpurun_out/lrpmc_c.log 2>&1 && echo PC_OK ;;
  *) echo "unknown kind $kind"; exit 2 ;;
esac
