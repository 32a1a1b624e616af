set -x
mkdir -p gpurun_out/r5y
python3 - <<'PY'
import sys, random
sys.path.insert(0, 'tests')
import _streams as S
w = S.c3_stream(random.Random(12), 100, frames_per_unit=1000)
open('/tmp/c3.bin', 'wb').write(w)
PY
timeout -k 10 120 node tests/js/decode_events.js /tmp/c3.bin 1048576 h2d 0 > gpurun_out/r5y/c3node.out 2> gpurun_out/r5y/c3node.err
echo "rc=$?" >> gpurun_out/r5y/c3node.err
true
