#!/bin/bash
# SQ counters per kernel for a short C2 decode (one rocprofv3 --pmc pass).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcs -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --frames 20000000 --steps 1 --warmup 0 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/pmcs.log 2>&1
