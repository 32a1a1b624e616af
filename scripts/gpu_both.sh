#!/bin/bash
# Parity suite on both decode kernels (speculative default, exact) + per-kernel timing of each.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_spec.log 2>&1
tail -1 gpurun_out/t_spec.log
DRP_DECODE=exact timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_exact.log 2>&1
tail -1 gpurun_out/t_exact.log
for M in spec exact; do
  cd /tmp
  DRP_DECODE=$M timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/k_$M -o run -- \
    python3 -u $GRAFT_REPO_ROOT/bench.py --frames ${1:-20000000} --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/k_$M.log 2>&1
  cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/k_$M -name "*kernel_stats.csv" | head -1)
  echo "== $M $(tail -1 gpurun_out/k_$M.log | cut -c1-200)"; cut -d, -f1-4 "$f" | grep "drp::" | cut -c1-110
done
