#!/bin/bash
# rocprofv3 kernel stats of the decode with ablated spec_claims builds (measurement only).
# Usage: gpurun -- 'bash scripts/gpu_ablate.sh "v1 v2" [frames | c5]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $1; do
  cd /tmp
  DRP_DECODE= DRP_LIB=$GRAFT_REPO_ROOT/exp/$v/libdrp.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/abl_$v -o run -- python3 -u $GRAFT_REPO_ROOT/scripts/time_claims.py ${2:-20000000} \
    > $GRAFT_REPO_ROOT/gpurun_out/abl_$v.log 2>&1
  cd $GRAFT_REPO_ROOT
  echo "$v done"
done
