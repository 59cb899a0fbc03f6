# Round-2 memory-hierarchy PMC passes + kernel trace on the CURRENT forest builder
# (feature-major large tier, bin scratch): 1M x 100, 5 fits x 100 trees (one bench batch).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
A="scripts/gbench_forest.py 1000000 100 100 5"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc3_kt -o p -- python3 $A > gpurun_out/pmc3_kt.log 2>&1 && echo KT_OK && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3_a -o p -- python3 $A > gpurun_out/pmc3_a.log 2>&1 && echo PA_OK && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3_b -o p -- python3 $A > gpurun_out/pmc3_b.log 2>&1 && echo PB_OK && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3_c -o p -- python3 $A > gpurun_out/pmc3_c.log 2>&1 && echo PC_OK && \
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc3_d -o p -- python3 $A > gpurun_out/pmc3_d.log 2>&1 && echo PD_OK
