#!/bin/bash
# A/B: misses (DRP_STATS capture) + spec kernel time per build. Usage: gpu_ab2.sh lib...
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in "$@"; do
  echo "== $L"
  DRP_LIB=$GRAFT_REPO_ROOT/$L DRP_STATS=1 DRP_TRACE=1 timeout -k 10 120 python -u bench.py --frames 20000000 --steps 1 --warmup 0 --no-cpu 2>&1 | grep "drp-spec" | head -1 | cut -c1-60
  cd /tmp
  DRP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab2_$(basename $L .so) -o run -- \
    python3 -u $GRAFT_REPO_ROOT/bench.py --frames 20000000 --steps 3 --warmup 1 --no-cpu > /dev/null 2>&1 || true
  cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/ab2_$(basename $L .so) -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-4 "$f" | grep "spec_claims\|verify_counts\|emit_tiles" | cut -c1-110
done
