# resumable refill (budget 6): full GPU suite, smoke, pool soak, benches, trace profile
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
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_b0 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --refill-budget 0
run bench_128 300 python bench.py --steps 128 --warmup 5 --no-cpu-baseline
run bench_mixed 300 python bench.py --systems 0,1,2,3 --steps 20 --warmup 5 --cpu-seconds 5
