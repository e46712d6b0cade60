# resumable refill: parity (pool tests, graph, restore), then bench A/B of the refill budget
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=4 run pytest_pool 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -k "pool or graph or state_dict or restore or refill or seed"
for i in 1 2; do
  for b in 6 0; do
    run bench_budget${b}_$i 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --refill-budget $b
  done
done
for b in 5 8; do
  run bench_budget${b} 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --refill-budget $b
done
run time_refill_budget 300 python tools/time_refill_budget.py 65536 0,4,5,6,7,8,10
