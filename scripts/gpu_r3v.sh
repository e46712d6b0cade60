# group-lane resets for the rigid RK4 model: full GPU suite, refill timing, configs[1] bench
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run refill_parts_rigid 120 python tools/time_refill_parts.py 4096 rigid
run refill_parts 120 python tools/time_refill_parts.py 65536
run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
run bench_c2b 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
run bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
