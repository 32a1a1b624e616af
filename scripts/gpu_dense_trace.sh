#!/bin/bash
# Kernel traces of one 1.7 GB dense two-framing cascade decode (scripts/probe_dense.py 1), with the
# default pointer-jumping threshold and with DRP_JUMP_MIN=0 (every unsettled tile jumps).
# Usage: gpurun -- 'bash scripts/gpu_dense_trace.sh <tag>'; timelines: scripts/trace_timeline.py
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$1/gated -o run -- python3 -u $R/scripts/probe_dense.py 1 > $R/gpurun_out/$1/gated.log 2>&1
DRP_JUMP_MIN=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$1/ungated -o run -- python3 -u $R/scripts/probe_dense.py 1 > $R/gpurun_out/$1/ungated.log 2>&1
echo "dense trace done"
