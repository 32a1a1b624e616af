#!/bin/bash
# CPU profile of the Node decode path (bench_node.js, C2 sample, 64 KiB writes) on the GPU box:
# node --cpu-prof into gpurun_out/<tag>/. Usage: gpurun -- 'bash scripts/gpu_node_prof.sh <tag>'
set -e
export DRP_DEBUG=1
OUT=gpurun_out/$1
mkdir -p $OUT
python3 -c "
import sys; sys.path.insert(0, 'tests'); import _streams as S
open('/tmp/c2_4m.bin', 'wb').write(S.c2_stream(4_000_000, seed=9).tobytes())"
DRP_MAX_BATCH=$((64 << 20)) timeout -k 10 300 node scripts/bench_node.js /tmp/c2_4m.bin 65536 3 > $OUT/node64k.json
DRP_MAX_BATCH=$((64 << 20)) timeout -k 10 300 node --cpu-prof --cpu-prof-dir $OUT scripts/bench_node.js /tmp/c2_4m.bin 65536 3 > $OUT/node64k_prof.json
DRP_MAX_BATCH=$((256 << 20)) timeout -k 10 300 node scripts/bench_node.js /tmp/c2_4m.bin 268435456 3 > $OUT/node256m.json
echo node prof done
