# Round-3 evidence refresh on HEAD: full GPU suite, smoke, pool soak, benches (headline x2,
# 128 steps, float64 obs, configs[1] x2, configs[4], mixed systems, two-rank gloo rehearsal).
set -o pipefail
mkdir -p gpurun_out
run() {   # run <name> <seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -${TAILN:-2} "gpurun_out/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "abnormal exit, stopping"; exit $rc; fi
}
TAILN=3 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_2 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
run bench_128 300 python bench.py --steps 128 --warmup 5 --no-cpu-baseline
run bench_obs64 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --obs-dtype float64
run bench_c2 300 python bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 5
run bench_c2b 300 python bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline
run bench_c5 300 python bench.py --config 5 --steps 20 --warmup 5 --cpu-seconds 5
run bench_mixed 300 python bench.py --systems 0,1,2,3 --steps 20 --warmup 5 --cpu-seconds 5
run bench_n2_gloo 300 env CTR_BENCH_BACKEND=gloo CTR_BENCH_SAME_DEVICE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline
