# HIP-graph replay of refill periods: parity, then benches with and without graphs
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-3} "gpurun_out/$name.log" | cut -c1-600
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=8 run pytest_graph 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread
run bench_c2_graph 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
run bench_c2_nograph 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline --graph off
run bench_graph 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_nograph 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --graph off
run bench_c5_graph 300 python bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline
