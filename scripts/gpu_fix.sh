#!/bin/bash
# Parity suite + C2 and C4 bench lines (deadlock regression check for the 8192-stream case).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c2.log 2>&1
timeout -k 10 240 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_c4.log 2>&1
