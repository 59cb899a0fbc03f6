set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
for v in v4_nt256 v4_nt512 v4_nt1024; do DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 200 python scripts/sweep_tiers.py > gpurun_out/ab4_$v.log 2>&1 || exit 1; echo "$v $(grep build gpurun_out/ab4_$v.log)"; done
DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/v4_nt1024.so timeout -k 10 300 python scripts/sweep_tiers.py block_max=16384,65536 wave_max=128,256 > gpurun_out/ab4_sweep.log 2>&1; grep build gpurun_out/ab4_sweep.log
