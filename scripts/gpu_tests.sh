#!/bin/bash
# GPU parity tests only. Usage: gpurun --timeout 600 -- 'bash scripts/gpu_tests.sh [pytest args]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" \
  > gpurun_out/gpu_tests.log 2>&1
