#!/bin/bash
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
DRP_STATS=1 DRP_TRACE=1 timeout -k 10 120 python -u bench.py --frames ${1:-2000000} --steps 1 --warmup 0 --no-cpu > gpurun_out/spec_dbg.log 2>&1
grep "drp-spec\|decode_spec" gpurun_out/spec_dbg.log | head -5
