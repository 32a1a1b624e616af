#!/bin/bash
# Per-kernel durations of a short C2 decode (rocprofv3 kernel trace). Usage: [frames]
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pq -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --frames ${1:-20000000} --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pq.log 2>&1
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/pq -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | grep -v "at::native" | head -12
