set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/time_refill_parts.py 4096 rigid > gpurun_out/refill_parts.log 2>&1 || exit 1
timeout -k 10 120 python tools/time_refill_parts.py 65536 >> gpurun_out/refill_parts.log 2>&1 || exit 2
timeout -k 10 120 python tools/time_refill_parts.py 4096 >> gpurun_out/refill_parts.log 2>&1 || exit 3
grep refill gpurun_out/refill_parts.log
