#!/bin/bash
# round 5: a kernel trace over the whole driver bench command (setup + warmup + timed steps)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
s=$(date +%s.%N)
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wholebench -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/wb_bench.log 2>&1 || exit 1
e=$(date +%s.%N)
tail -1 gpurun_out/wb_bench.log | cut -c1-200
python3 scripts/whole_run_busy.py gpurun_out/wholebench $(python3 -c "print($e-$s)") 5
rm -rf gpurun_out/wholebench
