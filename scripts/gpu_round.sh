#!/bin/bash
# Round measurement: PMC passes (speculative decode, 20M frames), full C2 bench, rocprofv3
# kernel stats of the same bench command, and the C4 multi-stream bench.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_pmc.sh 20000000
echo pmc done
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1
echo bench done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_prof.log 2>&1
cd $GRAFT_REPO_ROOT
echo prof done
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu > gpurun_out/bench_c4.log 2>&1
echo c4 done
