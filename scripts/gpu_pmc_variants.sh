#!/bin/bash
# FETCH/WRITE PMC passes of the decode per libdrp variant (scripts/build_variant.sh), on
# scripts/time_claims.py (no output check: measurement builds). Usage: gpurun -- 'bash scripts/gpu_pmc_variants.sh "v1 v2"'
set -e
mkdir -p gpurun_out/pmcv
export TMPDIR=/tmp
for v in $1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    DRP_LIB=exp/$v/libdrp.so timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcv/$v/$c -o run -- \
      python3 -u scripts/time_claims.py 20000000 > gpurun_out/pmcv/$v.$c.log 2>&1
  done
  echo "$v done"
done
