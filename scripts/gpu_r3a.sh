# Round 3, first GPU pass: the suite (with the copy-engine gather tests), the gather interference
# measurement with real copy-engine copies, the headline bench and the two-rank sdma rehearsal.
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-6} "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=4 run pytest_gather 300 python -u -m pytest tests/test_gpu_gather.py -x -v --timeout 120 --timeout-method thread
run interf_sdma8 240 python tools/gather_interference.py sdma 8 8
run interf_sdma8_s1 240 python tools/gather_interference.py sdma 8 1
run interf_sdma8_s4 240 python tools/gather_interference.py sdma 8 4
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_n2_sdma 300 env CTR_BENCH_BACKEND=gloo CTR_BENCH_SAME_DEVICE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
TAILN=12 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
