#!/bin/bash
# A/B of libdrp builds on the C5 round trip (decode ms, repairs, fallbacks) and a 20M-frame C2.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in "$@"; do
  DRP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/abc5_$(basename $L .so).log 2>&1
  DRP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python -u bench.py --frames 20000000 --steps 3 --warmup 1 --no-cpu > gpurun_out/abc2_$(basename $L .so).log 2>&1
  echo "== $L"
  grep -o '"encode": {[^}]*}\|"decode": {[^}]*}' gpurun_out/abc5_$(basename $L .so).log
  grep -o '"kernel_ms": [0-9.]*\|"exact_fallbacks": [0-9]*\|"repair_passes": [0-9]*' gpurun_out/abc2_$(basename $L .so).log | tr '\n' ' '; echo
done
