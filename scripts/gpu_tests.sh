#!/bin/bash
# GPU parity tests only. Usage: gpurun --timeout 900 -- 'bash scripts/gpu_tests.sh [tag] [pytest args]'
set -e
export TMPDIR=/tmp
TAG=${1:-run}
shift || true
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -m gpu -x -v --timeout 150 --timeout-method thread "${@:-tests}" \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
