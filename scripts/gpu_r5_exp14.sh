# Round-5 batch 14: LR forward item order (column groups of 2 / 4 tiles) vs row-tile-major.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=cs230_distributed_machine_learning_amd/lib
for v in cur cg2 cg4; do
  if [ $v = cur ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$v.so; fi
  DML_HIP_LIB=$lib timeout -k 10 200 python -u scripts/lr_kernel_bench.py 10000000 1000 2560 > gpurun_out/e19_lrk_$v.log 2>&1 || exit 1
  echo "$v: $(tail -1 gpurun_out/e19_lrk_$v.log)"
done
