#!/bin/bash
# SQ instruction counters of the decode for libdrp variants (exp/<v>/libdrp.so, built by
# scripts/build_variant.sh; DRP_ABLATE_F=N builds stop claims_fast after phase N) over
# scripts/time_claims.py (no result check).
# Usage: gpurun -- 'bash scripts/gpu_pmc_ablate.sh "v1 v2 ..." [frames]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
F=${2:-20000000}
for v in $1; do
  cd /tmp
  DRP_LIB=$GRAFT_REPO_ROOT/exp/$v/libdrp.so timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU \
    SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/pmcab/$v -o run -- python3 -u $GRAFT_REPO_ROOT/scripts/time_claims.py $F \
    > $GRAFT_REPO_ROOT/gpurun_out/pmcab/$v.log 2>&1 || { rc=$?; case $v in abl*|fa*) [ $rc = 1 ] || exit $rc;; *) exit $rc;; esac; }
  cd $GRAFT_REPO_ROOT
  echo "$v done"
done
