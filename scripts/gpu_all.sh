#!/bin/bash
# One GPU session: parity tests, smoke, the default bench line, the C5 round-trip bench and the
# rocprofv3 kernel-trace summary of the default bench command. Every GPU step has its own time
# limit; the first failure ends the script (set -e), so nothing runs on the GPU after a fault.
# Usage: gpurun --timeout 1200 -- 'bash scripts/gpu_all.sh [tag]'
set -e
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.log 2>&1
echo tests done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
echo smoke done
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
echo bench done
timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c5_$TAG.log 2>&1
echo c5 done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_prof_$TAG.log 2>&1
echo prof done
