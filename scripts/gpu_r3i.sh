# kernel trace of bench --config 2 (where the non-kernel time of a 13 us step goes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/trace_c2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2 -o run -- python3 bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/trace_c2/log.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/host_floor.py > gpurun_out/host_floor.log 2>&1 || exit 2
tail -5 gpurun_out/host_floor.log
