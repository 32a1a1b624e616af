set -e
export TMPDIR=/tmp
for v in $1; do
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_c5_$v.log 2>&1
  echo "$v done"
done
