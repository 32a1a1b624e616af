#!/bin/bash
# Round-3 session c: dense-cascade probe, the GPU suite, smoke, bench lines (C2 default, C5, C4),
# the kernel-trace summary, then the pipelined decode: a parity subset with tiny chunks (every
# stream of >= 1 MiB goes through it) and C2 bench lines at three chunk sizes.
set -e
export TMPDIR=/tmp
TAG=r3c
mkdir -p gpurun_out
DRP_TRACE=1 timeout -k 10 300 python -u scripts/probe_dense.py > gpurun_out/probe_dense.log 2> gpurun_out/probe_dense.err
echo probe done
bash scripts/gpu_session.sh $TAG "enc_old nt64" ""
DRP_PIPE_CHUNK=64 timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu \
  tests/test_gpu_decode.py tests/test_gpu_ref_fixtures.py tests/test_gpu_cascade.py tests/test_gpu_emit_split.py \
  tests/test_gpu_adversarial.py > gpurun_out/pipe_tests_$TAG.log 2>&1
echo pipe tests done
for ch in 8192 32768 131072; do
  DRP_PIPE_CHUNK=$ch timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/pipe_c2_$ch.log 2>&1
  echo "pipe $ch done"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_dense -o run -- \
  python3 -u $GRAFT_REPO_ROOT/scripts/probe_dense.py > $GRAFT_REPO_ROOT/gpurun_out/probe_dense_prof.log 2>&1)
echo dense prof done
