#!/bin/bash
# Round-3 session d: the GPU suite (failures reported, not fatal), smoke, bench lines (C2 default,
# C5, C4), the kernel-trace summary, A/B variants, and kernel traces of C5 and the dense probe. Each GPU step has its own limit; a crash or timeout ends it.
set -e
export TMPDIR=/tmp
TAG=${1:-r3d}
mkdir -p gpurun_out
bash scripts/gpu_session.sh $TAG "${2:-}" ""
(cd /tmp && DRP_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dense -o run -- \
  python3 -u $GRAFT_REPO_ROOT/scripts/probe_dense.py > $GRAFT_REPO_ROOT/gpurun_out/probe_dense_prof.log 2>&1)
echo dense prof done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_c5_prof.log 2>&1)
echo c5 prof done
timeout -k 10 400 python -u scripts/probe_c5_miss.py > gpurun_out/probe_c5.log 2>&1
echo c5 probe done
