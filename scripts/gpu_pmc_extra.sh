#!/bin/bash
# Extra PMC passes (instruction fetch, SALU cycles, LDS mix) over a C2 decode.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
F=${1:-20000000}
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc/$name -o run -- \
    python3 -u bench.py --frames $F --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc/$name.log 2>&1
}
run sqx SQ_IFETCH SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_ATOMIC SQ_IFETCH_LEVEL SQ_INSTS_VSKIPPED
run sqc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ
