# A/B: C3 through the pipelined staging at several DRP_PIPE_CHUNK (MiB; 0 = staged whole) / DRP_WALK_MIN values
set -o pipefail
mkdir -p gpurun_out/ab
for cfg in "64 32768" "64 4096" "128 8192" "128 32768" "256 32768" "0 32768"; do
  set -- $cfg
  DRP_PIPE_CHUNK=$1 DRP_WALK_MIN=$2 timeout -k 10 120 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu > gpurun_out/ab/c3_$1_$2.log 2>&1 || exit 1
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab/c3_$1_$2.log').read().strip().splitlines()[-1]);print('$1 $2',round(d['ms_per_step'],2),round(d['h2d']['ms'],2),round(d['d2h_ms'],2),round(d['roofline']['kernel_ms'],2))"
done
