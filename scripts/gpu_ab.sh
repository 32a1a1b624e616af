#!/bin/bash
# A/B kernel timing of two libdrp builds on the same box. Usage: gpu_ab.sh libA libB
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in "$@"; do
  cd /tmp
  DRP_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_$(basename $L .so) -o run -- \
    python3 -u $GRAFT_REPO_ROOT/bench.py --frames 20000000 --steps 3 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/ab_$(basename $L .so).log 2>&1 || true
  cd $GRAFT_REPO_ROOT
  f=$(find gpurun_out/ab_$(basename $L .so) -name "*kernel_stats.csv" | head -1)
  echo "== $L"; cut -d, -f1-4 "$f" | grep "spec::\|decode_tiles" | cut -c1-120
done
