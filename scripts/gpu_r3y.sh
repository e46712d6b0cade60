# carry sub-lists: pool/graph parity, refill timing, clock-stamped phases (refill + k_step)
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=3 run pytest_pool 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -k "pool or graph or state_dict or restore or refill or seed"
run time_refill_budget 300 python tools/time_refill_budget.py 65536 0,6,8
TAILN=20 run diag 120 env CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_diag.so python tools/diag_refill.py 6
run bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
