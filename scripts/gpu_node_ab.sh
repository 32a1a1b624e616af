#!/bin/bash
# Node decode path A/B on one box: this tree's package vs the one under $1 (a built package
# directory), 64 KiB and 256 MiB writes, alternating. Usage: gpu_node_ab.sh <other pkg> <tag>
set -e
export DRP_DEBUG=1
OUT=gpurun_out/$2
mkdir -p $OUT
python3 -c "
import sys; sys.path.insert(0, 'tests'); import _streams as S
open('/tmp/c2_4m.bin', 'wb').write(S.c2_stream(4_000_000, seed=9).tobytes())"
for r in 1; do
  for v in cur other; do
    if [ $v = other ]; then P=$(realpath $1); else P=$(realpath dat-replication-protocol_amd); fi
    DRP_PKG=$P DRP_MAX_BATCH=$((64 << 20)) timeout -k 10 300 node scripts/bench_node.js /tmp/c2_4m.bin 65536 3 > $OUT/${v}_64k_$r.json
    DRP_PKG=$P DRP_MAX_BATCH=$((256 << 20)) timeout -k 10 300 node scripts/bench_node.js /tmp/c2_4m.bin 268435456 3 > $OUT/${v}_256m_$r.json
  done
done
echo node ab done
