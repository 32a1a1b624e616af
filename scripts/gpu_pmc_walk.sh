#!/bin/bash
# SQ counter passes of the C2 decode (20M frames) for the claims kernels: instruction mix, wave
# cycles and waits (one rocprofv3 run per pass). Usage: gpurun -- 'bash scripts/gpu_pmc_walk.sh <outdir> [K=V ...]'
set -e
export TMPDIR=/tmp
D=$1; shift
for kv in "$@"; do export "$kv"; done
mkdir -p $D
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $D/$name -o run -- \
    python3 -u bench.py --frames 20000000 --workload c2 --steps 1 --warmup 1 --no-cpu --no-sub > $D/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH
run sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT
run sq3 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU
