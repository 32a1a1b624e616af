#!/bin/bash
# Speculative decode bring-up: smoke, a traced C2 bench, then the GPU parity suite.
# Usage: gpurun --timeout 600 -- 'bash scripts/gpu_spec.sh [frames]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
F=${1:-20000000}
timeout -k 10 60 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
DRP_TRACE=1 timeout -k 10 180 python -u bench.py --frames $F --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_spec.log 2>&1
grep -c "prediction failed" gpurun_out/bench_spec.log || true
tail -1 gpurun_out/bench_spec.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -3 gpurun_out/gpu_tests.log
