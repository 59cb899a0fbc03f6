# Round-5 batch 7: tier stream priority / block-first launch order A/B (sweep build), LR PMC roofline passes.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in cur p001 bf p001bf p011; do
  case $v in cur) E="";; p001) E="DML_TIER_PRIO=001";; bf) E="DML_BLOCK_FIRST=1";; p001bf) E="DML_TIER_PRIO=001 DML_BLOCK_FIRST=1";; p011) E="DML_TIER_PRIO=011";; esac
  env $E timeout -k 10 300 python -u scripts/sweep_tiers.py > gpurun_out/e11_$v.log 2>&1 || exit 1
  echo "$v: $(grep build gpurun_out/e11_$v.log | cut -c1-60)"
done
A=10000000; 
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/e11_lra -o p -- python3 scripts/lr_kernel_bench.py $A 1000 2560 > gpurun_out/e11_lra.log 2>&1 && echo PA_OK && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/e11_lrb -o p -- python3 scripts/lr_kernel_bench.py $A 1000 2560 > gpurun_out/e11_lrb.log 2>&1 && echo PB_OK && \
timeout -s KILL 200 rocprofv3 --pmc TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/e11_lrc -o p -- python3 scripts/lr_kernel_bench.py $A 1000 2560 > gpurun_out/e11_lrc.log 2>&1 && echo PC_OK
