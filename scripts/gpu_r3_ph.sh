# Philox as 64-bit products + refill staging preload: GPU suite, refill phase stamps, refill timing, benches
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
TAILN=20 run diag_refill 200 env CTR_REACH_AMD_LIB=$PWD/gym-ctr-reach_amd/ctr_reach_amd/lib/libab_diag.so python tools/diag_refill.py 6
TAILN=6 run time_refill_budget 300 python tools/time_refill_budget.py 65536 0,6
run bench 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
run bench_c2b 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
