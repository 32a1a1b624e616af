#!/bin/bash
# C5 round trip under rocprofv3 kernel stats, plus the C3 test.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -k "c3 or c5" > gpurun_out/c3c5_test.log 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/bench_c5_prof.log 2>&1
