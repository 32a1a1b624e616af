#!/bin/bash
# PMC counter passes over one workload's decode (one rocprofv3 run per pass, as the pool requires).
# Usage: gpurun --timeout 900 -- 'bash scripts/gpu_pmc.sh [frames] [c2|c3|c4|c5] [outdir]'; summary:
# scripts/pmc_kernels.py (c5: the C5 round trip, 1M Changes: encode + decode kernels; c4: 8192 streams)
set -e
export TMPDIR=/tmp
F=${1:-20000000}
W=${2:-c2}
D=${3:-gpurun_out/pmc}
mkdir -p $D
# (c3: the HBM-resident decode of a ~1 GiB C3 stream that prices the C3 roofline (bench.py
# --c3-leg device), warmup 1 + 1 step = 2 decode calls: pmc_kernels.py --calls 2 divides the
# kernels' totals by 2 x the stream's frames)
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $D/$name -o run -- \
    python3 -u bench.py --frames $F --workload $W --steps 1 --warmup 1 --no-cpu --no-sub --no-after-c2 $([ $W = c3 ] && echo --c3-leg device) > $D/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH
run sq2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_FLAT
run fetch FETCH_SIZE
run write WRITE_SIZE
