# A/B: the repair's dirty-list run limit (DRP_DIRTY_RUN) on the HBM-resident C3 decode, with
# DRP_TRACE's pass lines; exp/<v>/libdrp.so from scripts/build_variant.sh
set -o pipefail
mkdir -p gpurun_out/dr
for v in "$@"; do
  DRP_TRACE=1 DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c3 --c3-leg device --steps 5 --warmup 1 --no-cpu > gpurun_out/dr/$v.log 2> gpurun_out/dr/$v.err || exit 1
  echo "$v $(tail -1 gpurun_out/dr/$v.log | cut -c1-60) $(grep -m3 'passes' gpurun_out/dr/$v.err | tr '\n' ';')"
  DRP_LIB=exp/$v/libdrp.so timeout -k 10 200 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu > gpurun_out/dr/${v}_host.log 2>&1 || exit 1
  echo "$v host: $(tail -1 gpurun_out/dr/${v}_host.log | cut -c1-110)"
done
