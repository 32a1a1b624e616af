#!/bin/bash
# Build libdrp with extra compile definitions into exp/<name>/libdrp.so (A/B experiments;
# select with DRP_LIB=exp/<name>/libdrp.so). Usage: scripts/build_variant.sh <name> [-DFOO=1 ...]
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/exp/$NAME
mkdir -p $OUT/build
SRCS="drp_decode drp_decode_spec drp_walk drp_encode drp_keys drp_comm drp_api"
FLAGS="-O3 -std=c++17 -fPIC -fvisibility=hidden -fno-strict-aliasing --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value $*"
pids=""
for s in $SRCS; do
  /opt/rocm/bin/hipcc $FLAGS -c $ROOT/dat-replication-protocol_amd/csrc/$s.hip -o $OUT/build/$s.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc $FLAGS -shared -o $OUT/libdrp.so $OUT/build/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $OUT/libdrp.so
