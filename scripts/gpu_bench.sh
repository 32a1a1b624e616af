#!/bin/bash
# Bench + rocprofv3 kernel-trace summary on the GPU box.
# Usage: gpurun --timeout 900 -- 'bash scripts/gpu_bench.sh [extra bench args]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 "$@" > gpurun_out/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 -u bench.py --steps 5 --warmup 2 --no-cpu "$@" > gpurun_out/bench_prof.log 2>&1
