set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_kt -o kt -- python scripts/gbench_forest.py 1000000 100 20 5 > gpurun_out/pmc_kt.log 2>&1 && echo KT_OK && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc1 -o p1 -- python scripts/gbench_forest.py 1000000 100 20 5 > gpurun_out/pmc1.log 2>&1 && echo P1_OK && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc2 -o p2 -- python scripts/gbench_forest.py 1000000 100 20 5 > gpurun_out/pmc2.log 2>&1 && echo P2_OK
