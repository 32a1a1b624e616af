#!/bin/bash
# Round-3 session q: GPU suite and smoke on the final build, then the FETCH_SIZE / WRITE_SIZE
# passes of a 20M-frame C2 decode (one rocprofv3 run per pass). Any failure ends the script.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_q
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -rA --timeout 150 --timeout-method thread \
  > gpurun_out/gpu_tests_q2.log 2>&1
echo tests done
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_q2.log 2>&1
echo smoke done
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d gpurun_out/pmc_q/$pass -o run -- \
    python3 -u bench.py --frames 20000000 --workload c2 --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc_q/$pass.log 2>&1
  echo "$pass done"
done
