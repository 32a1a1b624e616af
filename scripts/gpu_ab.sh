#!/bin/bash
# A/B of libdrp variants built by scripts/build_variant.sh: C2 (100M frames) and C5 benches per
# variant, optional parity subset. Usage: gpurun -- 'bash scripts/gpu_ab.sh "v1 v2 ..." [test]'
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in $1; do
  if [ "$2" = "test" ]; then
    DRP_LIB=exp/$v/libdrp.so timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 150 --timeout-method thread \
      tests/test_gpu_decode.py tests/test_gpu_adversarial.py tests/test_gpu_multistream.py tests/test_gpu_ref_fixtures.py \
      > gpurun_out/ab_test_$v.log 2>&1
    echo "$v tests ok"
  fi
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_c2_$v.log 2>&1
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_c5_$v.log 2>&1
  echo "$v bench done"
done
