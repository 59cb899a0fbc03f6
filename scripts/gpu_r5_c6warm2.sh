#!/bin/bash
# round 5: why a warmup fit slows config 6 -- phase summaries and idle gaps with / without it
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in 1 0; do
  DML_C6_WARMUP=$w timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cw2_c6_$w.log 2>&1 || exit 1
  echo "[warmup=$w] $(grep '^{' gpurun_out/cw2_c6_$w.log | cut -c1-1500)"
done
DML_C6_WARMUP=1 DML_ARENA_LOG=1 timeout -k 10 300 python -u scripts/bench_configs.py --configs 6 > gpurun_out/cw2_arena.log 2>&1 || exit 1
grep -i "arena" gpurun_out/cw2_arena.log | head -20
