set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof12 -o b -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof12.log 2>&1 && echo PROF_OK
