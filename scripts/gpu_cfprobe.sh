#!/bin/bash
# C5 claims cost with and without the long-frame check (DRP_CHANGE_CHECKS forces the claims form)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/cf
for cc in 1 0; do
  (cd /tmp && DRP_CHANGE_CHECKS=$cc timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/cf/cc$cc -o run -- \
    python3 -u $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/cf/c5_cc$cc.log 2>&1)
  echo cc$cc done
done
