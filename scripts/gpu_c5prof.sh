#!/bin/bash
# C5 round trip under rocprofv3 kernel stats.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/bench_c5_prof.log 2>&1
