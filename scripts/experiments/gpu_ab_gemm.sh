set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
for v in g0_base g1_pass1 g2_noload g3_nostore g4_nomfma g5_noload_nostore; do DML_HIP_LIB=$PWD/variants/$v.so timeout -k 10 120 python scripts/lr_kernel_bench.py > gpurun_out/abg_$v.log 2>&1 || exit 1; tail -1 gpurun_out/abg_$v.log; done
