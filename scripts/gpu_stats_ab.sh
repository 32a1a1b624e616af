#!/bin/bash
# DRP_STATS=1 decode (misses, link rounds, per-phase cycles) for libdrp variants.
# Usage: gpurun -- 'bash scripts/gpu_stats_ab.sh "v1 v2 ..." [frames] [workload]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
F=${2:-20000000}
W=${3:-c2}
for v in $1; do
  DRP_LIB=exp/$v/libdrp.so DRP_STATS=1 timeout -k 10 200 python -u bench.py --frames $F --workload $W --steps 1 \
    --warmup 1 --no-cpu > gpurun_out/stats_${v}_$W.log 2>&1
  echo "$v done"
done
