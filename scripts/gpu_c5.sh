#!/bin/bash
# C5 round trip (encode -> decode, 1M Changes x 4 KB), the GPU parity suite, the C2 bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/bench_c5.log 2>&1
echo c5 done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo tests done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1
echo bench done
