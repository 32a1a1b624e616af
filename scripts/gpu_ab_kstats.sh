#!/bin/bash
# Interleaved A/B (two rounds) of libdrp variants plus a rocprofv3 kernel-stats pass of C2 per
# variant. Usage: gpurun -- 'bash scripts/gpu_ab_kstats.sh "v1 v2 ..."'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in $1; do
    DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_c2_${v}_r$r.log 2>&1
    DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_c5_${v}_r$r.log 2>&1
    echo "$v round $r done"
  done
done
for v in $1; do
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abk_$v -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/abk_$v.log 2>&1
  echo "$v kstats done"
done
