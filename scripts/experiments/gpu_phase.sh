set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
for v in rpt4_prof rpt1_prof; do DML_HIP_LIB=$GRAFT_REPO_ROOT/variants/$v.so timeout -k 10 200 python scripts/phase_prof.py > gpurun_out/phase_$v.log 2>&1 || exit 1; echo "== $v"; grep -v amdgpu.ids gpurun_out/phase_$v.log; done
