# A/B of encoder variants (exp/<v>/libdrp.so built with other DRP_ENC_* values) vs the build, C5
# Usage: bash scripts/ab_enc_dpp.sh v1 v2 ...   (then the GPU encode tests on the last variant)
set -o pipefail
mkdir -p gpurun_out/encab
for r in 1 2; do
  for v in base "$@"; do
    L=""; [ $v != base ] && L=exp/$v/libdrp.so
    DRP_LIB=$L timeout -k 10 200 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu > gpurun_out/encab/c5_${v}_$r.log 2>&1 || exit 1
    python3 -c "
import json;d=json.loads(open('gpurun_out/encab/c5_${v}_$r.log').read().strip().splitlines()[-1]);print('$v',d['ms_per_step'],d['encode']['ms'],d['decode']['ms'])"
  done
done
