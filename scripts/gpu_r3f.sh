set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
run bench_n2_auto 300 env CTR_BENCH_BACKEND=gloo CTR_BENCH_SAME_DEVICE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
TAILN=4 run pytest_cfg 600 python -u -m pytest tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread
