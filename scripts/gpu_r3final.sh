#!/bin/bash
# Round-3 final session: the GPU suite, smoke, bench lines (C2 default with the CPU baselines and
# the Node path, C5, C4), kernel-trace summaries (C2, C5, dense cascade probe), then the PMC passes
# of a 20M-frame C2 decode (FETCH_SIZE / WRITE_SIZE / SQ counters, one pass each).
set -e
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out
bash scripts/gpu_session.sh $TAG "${2:-}" ""
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run -- \
  python3 -u $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/bench_c5_prof.log 2>&1)
echo c5 prof done
(cd /tmp && DRP_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dense -o run -- \
  python3 -u $GRAFT_REPO_ROOT/scripts/probe_dense.py > $GRAFT_REPO_ROOT/gpurun_out/probe_dense_prof.log 2>&1)
echo dense prof done
bash scripts/gpu_pmc.sh 20000000 c2
echo pmc done
# two ranks on the box's one GPU over gloo (the RCCL path is the driver's 8-GPU run): C5 round trip
# and C4 stream shards with the stats all-gather and global index
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --workload c5 --steps 3 --warmup 1 --no-cpu \
  > gpurun_out/bench_c5_gloo2.log 2>&1
echo c5 gloo2 done
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --workload c4 --steps 3 --warmup 1 --no-cpu \
  > gpurun_out/bench_c4_gloo2.log 2>&1
echo c4 gloo2 done
