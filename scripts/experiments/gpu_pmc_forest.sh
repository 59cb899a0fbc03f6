# PMC passes on the forest builder microbench (20 fits x 125 trees would be the bench; 5 x 100 here).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
A="scripts/gbench_forest.py 1000000 100 100 5"
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1; \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_f1 -o p -- python3 $A > gpurun_out/pmc_f1.log 2>&1 && echo P1_OK && \
timeout -s KILL 150 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_f2 -o p -- python3 $A > gpurun_out/pmc_f2.log 2>&1 && echo P2_OK
