# PMC passes (one counter group per run) on the LR objective microbench.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="scripts/lr_objective_bench.py --rows 2000000 --features 1000 --fits 512 --reps 2"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_lro1 -o p -- python3 $A > gpurun_out/pmc_lro1.log 2>&1 && echo P1_OK && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/pmc_lro2 -o p -- python3 $A > gpurun_out/pmc_lro2.log 2>&1 && echo P2_OK
