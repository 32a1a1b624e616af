#!/bin/bash
# Parity tests per libdrp variant (exp/<v>/libdrp.so), all failures listed.
# Usage: gpurun -- 'bash scripts/gpu_ab_tests.sh "v1 v2 ..." [test files]'
export TMPDIR=/tmp
mkdir -p gpurun_out
V=$1; shift
for v in $V; do
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 150 --timeout-method thread \
    ${@:-tests/test_gpu_decode.py} > gpurun_out/abt_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"
  case $rc in 0|1) ;; *) exit $rc;; esac
done
