# Round-5 batch 18: GBRT config 6: HEAD library vs working tree, feature group 16 / 24.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=cs230_distributed_machine_learning_amd/lib
for rep in 1 2; do
for v in "head 16" "head 24" "cur 16" "cur 24"; do
  set -- $v
  if [ $1 = cur ]; then lib=$L/libdml_hip.so; else lib=$L/libdml_hip_$1.so; fi
  DML_HIP_LIB=$lib DML_TIER_KG_LARGE_REG=$2 timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/e23_c6.log 2>&1 || exit 1
  echo "[$1 kg=$2] $(grep -o '"cv_fits_per_s[^,]*' gpurun_out/e23_c6.log)"
done
done
