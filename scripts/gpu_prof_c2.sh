#!/bin/bash
# rocprofv3 kernel stats of a short C2 bench line (WORKLOAD=c4|c5: that one; no sub-lines, no CPU legs)
# into gpurun_out/<tag>/prof_<name>.
# Usage: gpurun -- 'bash scripts/gpu_prof_c2.sh <tag> <name> [env K=V ...]'
set -e
export TMPDIR=/tmp
TAG=$1; NAME=$2; shift 2
for kv in "$@"; do export "$kv"; done
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$NAME -o run -- \
  python3 -u $ROOT/bench.py --workload ${WORKLOAD:-c2} --steps 5 --warmup 2 --no-cpu --no-sub > $OUT/bench_$NAME.log 2>&1
python3 $ROOT/scripts/kstats.py $(find $OUT/prof_$NAME -name "*kernel_stats.csv" | head -1) > $OUT/kstats_$NAME.txt 2>&1 || true
echo "prof $NAME done: $(tail -1 $OUT/bench_$NAME.log | cut -c1-200)"
