#!/bin/bash
# One GPU session (round 3): parity suite, smoke, default bench line, C5 bench, rocprofv3 summary
# of the default bench, then optional experiments (A/B variants from exp/, the L3 probe). Each GPU
# step has its own limit; the first failure ends the script, nothing runs after a fault.
# Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_session.sh <tag> [ab variants] [l3]'
set -e
export TMPDIR=/tmp
TAG=${1:-run}
AB=${2:-}
mkdir -p gpurun_out
# test failures (rc 1) do not stop the session; a timeout, abort or crash (any other rc) does
set +e
timeout -k 10 700 python -u -m pytest tests -m gpu --maxfail=8 -v -rA --timeout 150 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
set -e
echo "tests done rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
echo smoke done
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
echo bench done
timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c5_$TAG.log 2>&1
echo c5 done
timeout -k 10 200 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c4_$TAG.log 2>&1
echo c4 done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1)
echo prof done
for v in $AB; do
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/ab_c2_$v.log 2>&1
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_c5_$v.log 2>&1
  echo "$v bench done"
done
