# One parameterised GPU experiment command (replaces the round-1 one-off files).
#   gpurun -- bash scripts/gpu_exp.sh <kind> [args...]
# kinds:
#   bench [bench.py args]        headline bench, JSON line to gpurun_out/exp_bench.log
#   prof  [bench.py args]        rocprofv3 kernel stats of bench.py  -> gpurun_out/exp_prof/
#   pmc   "<counters>" [gbench args]   one PMC pass on scripts/gbench_forest.py -> gpurun_out/exp_pmc/
#   sweep [sweep_tiers.py args]  forest tier sweep
#   configs [bench_configs.py args]   BASELINE configs 1/2/4/5
#   gbench [gbench_forest.py args]    forest builder micro-bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
kind=$1; shift
case "$kind" in
  bench)   timeout -k 10 900 python -u bench.py "$@" > gpurun_out/exp_bench.log 2>&1 && tail -1 gpurun_out/exp_bench.log ;;
  prof)    timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/exp_prof -o run -- python3 bench.py "$@" > gpurun_out/exp_prof.log 2>&1 && echo PROF_OK ;;
  pmc)     ctrs=$1; shift; args=${*:-1000000 100 100 5}
           timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/exp_pmc -o p -- python3 scripts/gbench_forest.py $args > gpurun_out/exp_pmc.log 2>&1 && echo PMC_OK ;;
  sweep)   timeout -k 10 900 python -u scripts/sweep_tiers.py "$@" > gpurun_out/exp_sweep.log 2>&1 && cat gpurun_out/exp_sweep.log ;;
  configs) timeout -k 10 900 python -u scripts/bench_configs.py "$@" > gpurun_out/exp_configs.log 2>&1 && cat gpurun_out/exp_configs.log ;;
  gbench)  timeout -k 10 600 python -u scripts/gbench_forest.py "$@" > gpurun_out/exp_gbench.log 2>&1 && cat gpurun_out/exp_gbench.log ;;
  *) echo "unknown kind $kind"; exit 2 ;;
esac
