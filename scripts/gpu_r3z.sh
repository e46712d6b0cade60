# staging loads ahead of the env rows, finish inputs parked in LDS, carry sub-lists: full GPU
# suite, smoke, pool soak, refill timing, benches (headline x2, configs[1] x2, 128 steps)
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
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=12 run soak_pool 600 python tools/soak_pool.py
run time_refill_budget 300 python tools/time_refill_budget.py 65536 0,6
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 5
run bench_c2b 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
run bench_128 300 python bench.py --steps 128 --warmup 5 --no-cpu-baseline
