# rocprofv3 kernel stats + one PMC pass of the LR objective microbench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lrobj -o o -- python3 scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 > gpurun_out/prof_lrobj.log 2>&1 && echo PROF_OK && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc_lrobj -o p -- python3 scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 --reps 2 > gpurun_out/pmc_lrobj.log 2>&1 && echo PMC_OK
