#!/bin/bash
# Infinity-Cache probe: per-kernel times of the C2 decode when the whole working set (wire +
# columns) fits in the 256 MiB L3 (frames small) against the full 100M-frame stream, so the
# gain of an L3-resident second pass over the wire can be read off before building a windowed
# pipeline. Usage: gpurun -- 'bash scripts/gpu_l3probe.sh [tag]'
set -e
export TMPDIR=/tmp
TAG=${1:-l3}
mkdir -p gpurun_out
cd /tmp
for F in 1000000 1500000 3000000 100000000; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_$F -o run -- \
    python3 -u $GRAFT_REPO_ROOT/bench.py --frames $F --steps 20 --warmup 3 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_$F.log 2>&1
  echo "frames $F done"
done
