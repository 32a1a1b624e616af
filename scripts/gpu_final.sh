#!/bin/bash
# Round-end measurement: GPU parity suite, C2 bench (with CPU baseline), rocprofv3 kernel stats
# of the same bench, C4 and C5 benches.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo tests done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
echo bench done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1
cd $GRAFT_REPO_ROOT
echo prof done
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c4.log 2>&1
echo c4 done
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/bench_c5.log 2>&1
echo c5 done
