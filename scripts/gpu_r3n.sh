#!/bin/bash
# Round-3 session n: PMC passes of the final build's C2 decode, then A/B lines: the encode write
# kernel's grid (C5) and the segmented repair's segment count (dense cascade probe).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_pmc.sh 20000000 c2
echo pmc done
timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_c5_base.log 2>&1
for v in enc_g32k enc_g256k; do
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu \
    > gpurun_out/ab_c5_$v.log 2>&1
  echo "$v done"
done
timeout -k 10 300 python -u scripts/probe_dense.py > gpurun_out/dense_base.log 2>&1
for v in seg4k seg8k; do
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 300 python -u scripts/probe_dense.py > gpurun_out/dense_$v.log 2>&1
  echo "$v done"
done
