set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
for v in old v3_w1 v3_w4 v3_w5; do DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 200 python scripts/sweep_tiers.py > gpurun_out/ab3_$v.log 2>&1 || exit 1; echo "$v $(grep build gpurun_out/ab3_$v.log)"; done
