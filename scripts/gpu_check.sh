#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Usage (from this container): gpurun --timeout 1100 -- 'bash scripts/gpu_check.sh'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python3 -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_prof.log 2>&1
