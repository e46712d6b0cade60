# kernel trace of the push-kernel interference run (do k_step and k_gather_push overlap?)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/trace_push
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_push -o run -- python3 tools/gather_interference.py push 8 32 > gpurun_out/trace_push/log.txt 2>&1 || exit 1
find gpurun_out/trace_push -name "*.csv" | head
