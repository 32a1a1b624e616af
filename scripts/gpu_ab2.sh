#!/bin/bash
# A/B of libdrp variants (exp/<v>/libdrp.so from scripts/build_variant.sh): C2 and C5 bench lines
# per variant. Usage: gpurun -- 'bash scripts/gpu_ab2.sh "v1 v2 ..." [tag]'
set -e
export TMPDIR=/tmp
TAG=${2:-ab}
mkdir -p gpurun_out
for v in $1; do
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/${TAG}_c2_$v.log 2>&1
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_c5_$v.log 2>&1
  echo "$v done"
done
