#!/bin/bash
# Decode timing (and DRP_STATS=1 event counters) on a C2 sample.
# Usage: gpurun -- 'bash scripts/gpu_stats.sh [frames] [waves_per_cu...]'
set -e
mkdir -p gpurun_out
F=${1:-2000000}
shift || true
WS=${@:-"16 8 4"}
for W in $WS; do
  DRP_WAVES_PER_CU=$W timeout -k 10 120 python -u bench.py --frames $F --steps 3 --warmup 1 --no-cpu \
    > gpurun_out/time_w$W.log 2>&1
  DRP_STATS=1 DRP_WAVES_PER_CU=$W timeout -k 10 120 python -u bench.py --frames $F --steps 1 --warmup 1 --no-cpu \
    > gpurun_out/stats_w$W.log 2>&1
done
