#!/bin/bash
# Per-phase cycle counts of the speculative kernels (DRP_STATS=1, thread 0 of each tile).
# Usage: gpurun -- 'bash scripts/gpu_stats.sh [frames] [workload]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
F=${1:-20000000}
W=${2:-c2}
DRP_STATS=1 timeout -k 10 200 python -u bench.py --frames $F --workload $W --steps 1 --warmup 1 --no-cpu \
  > gpurun_out/stats_$W.log 2>&1
