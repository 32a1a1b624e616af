set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o run -- python3 -u bench.py --frames 20000000 --steps 1 --warmup 1 --no-cpu > gpurun_out/pmc/fetch.log 2>&1
